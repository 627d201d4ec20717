#!/bin/bash
# FETCH_SIZE calibration for k_count's scattered 16-B reads (tools/fetch_calib.hip).
#   bash tools/fetch_calib.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-fcal}; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o /tmp/fetch_calib || exit 1
for m in 0 1 2; do
  run 60 rocprofv3 --pmc FETCH_SIZE -d $O/m$m -o m$m --output-format csv -- /tmp/fetch_calib $m > $O/m$m.log 2>&1
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for m in range(3):
    f = glob.glob(f"{o}/m{m}/**/*counter_collection.csv", recursive=True)[0]
    v = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            v[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    fetch = [x * 1024 for _, x in sorted(v.items())]
    line = open(f"{o}/m{m}.log").read().split("whole lines)")[0]
    lines = int(line.split("lines touched ")[1].split()[0])
    print(f"mode {m}: FETCH_SIZE bytes per dispatch {[int(x) for x in fetch]}; lines x 128 B = {lines * 128}; "
          f"ratio {fetch[-1] / (lines * 128):.3f}")
PY
