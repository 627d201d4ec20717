"""Table of kernel_ms / hbm_frac from an A/B directory: python tools/abtab.py gpurun_out/X"""
import glob, json, os, sys, collections
rows = collections.defaultdict(list)
for p in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    name = os.path.basename(p)[:-5].rsplit("_", 1)[0] if p.endswith(("_1.json", "_2.json", "_3.json")) else os.path.basename(p)[:-5]
    try:
        d = json.load(open(p))
        rows[name].append(f"{d['kernel_ms']:.3f}ms/{d['hbm_frac']:.3f}")
    except (ValueError, KeyError):
        rows[name].append("ERR")
for k, v in rows.items():
    print(f"{k:24s} {'  '.join(v)}")
