"""Per-step kernel time split of tools/r02_ktrace.sh output (span workloads):
python tools/kttab.py gpurun_out/PREFIX_ NAME..."""
import csv, glob, sys
pre = sys.argv[1]
for v in sys.argv[2:]:
    for w in ("config2r", "config3", "config5"):
        fs = glob.glob(f"{pre}{v}/{w}/**/kt_kernel_stats.csv", recursive=True)
        if not fs:
            print(v, w, "missing"); continue
        tot, parts = 0.0, []
        for r in csv.DictReader(open(fs[0])):
            n = r["Name"]
            if not ("mcrc" in n or "rocprim::ROCPRIM_400200" in n):
                continue
            if w == "config5" and ("k_final<0, false>" in n or "k_spans<false>" in n or "k_blocks<true" in n):
                continue  # (the bench's own setup: stored CRCs of the pages)
            t = float(r["TotalDurationNs"]) / 7 / 1000
            tot += t
            short = n.split("(")[0].replace("void ", "").replace("mcrc_dev::", "")[:22]
            parts.append(f"{short}={t:.0f}")
        print(v, w, f"total={tot:.0f}us", " ".join(parts))
