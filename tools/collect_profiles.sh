#!/bin/bash
# Copy one round's GPU evidence from gpurun_out/<round> into profiles/ (tracked).
set -e
R=${1:-r01}
O=gpurun_out/$R
P=profiles
cp $O/pytest_gpu.log $P/${R}_pytest_gpu.log
cp $O/bench.json $P/${R}_bench.json
[ -f $O/bench_default.json ] && cp $O/bench_default.json $P/${R}_bench_default.json
cp $O/kt/kt_kernel_stats.csv $P/${R}_bench_kernel_stats.csv
cp $O/traffic.json $P/${R}_traffic.json
cp $O/kt_c3/c3_kernel_stats.csv $P/${R}_config3_kernel_stats.csv
cp $O/kt_c5/c5_kernel_stats.csv $P/${R}_config5_kernel_stats.csv
python3 - "$O/x" "$P/${R}_extra_workloads.jsonl" <<'PY'
import glob, json, os, sys
src, dst = sys.argv[1], sys.argv[2]
with open(dst, "w") as f:
    for p in sorted(glob.glob(os.path.join(src, "*.json"))):
        try:
            f.write(json.dumps(json.load(open(p))) + "\n")
        except ValueError:
            pass
PY
ls -la $P
