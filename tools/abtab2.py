"""Table of tools/s3_ab.sh output: kernel_ms per variant, workload and rep.
    python tools/abtab2.py gpurun_out/DIR"""
import glob, json, os, re, sys
rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_*_*.json"))):
    m = re.match(r"(.+)_([a-z0-9]+)_(\d+)\.json$", os.path.basename(f))
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    v = d.get("kernel_ms") or (d.get("roofline") or {}).get("kernel_ms") or d.get("stamp_wbuf_us")
    rows.setdefault((m.group(2), m.group(1)), []).append(v)
for (w, v), ks in sorted(rows.items()):
    print(f"{w:10s} {v:8s} " + " ".join(f"{k:.3f}" for k in ks))
