"""Per-dispatch PMC values of the span kernel (k_spans) from tools/r02_pmc.sh output:
python tools/pmctab.py gpurun_out/X [kernel_substr]"""
import csv, glob, os, sys, collections
root = sys.argv[1]
ks = sys.argv[2] if len(sys.argv) > 2 else "k_spans"
for d in sorted(glob.glob(os.path.join(root, "*_[ab]"))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        vals = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if ks in r["Kernel_Name"]:
                vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        out = {c: sum(v.values()) / len(v) for c, v in vals.items()}
        print(os.path.basename(d), "  ".join(f"{c}={x:.4g}" for c, x in sorted(out.items())))
