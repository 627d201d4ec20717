"""HBM traffic per batch of the span workloads (config 3, config 5, stamps,
pages of mixed items) from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs: every
library kernel dispatched from the first batch on, summed per batch, against
the algorithmic bytes.  A batch starts at its first kernel (FIRST: k_census for
K5-routed item batches, k_count for planned span batches); the dispatches
before the first batch (the bench's own setup: the stored CRCs of the pages)
are not counted.  gfx950 correction as tools/traffic.py (FETCH_SIZE x 2, KiB).
    python tools/traffic_spans.py FETCH_DIR WRITE_DIR ALGO_BYTES OUT [FIRST]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_kernel(d, counter, first):
    rows = [r for r in csv.DictReader(open(glob.glob(f"{d}/*counter_collection.csv")[0]))
            if "mcrc" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    start = min(int(r["Dispatch_Id"]) for r in rows if first in r["Kernel_Name"])
    tot, calls = defaultdict(float), defaultdict(set)
    for r in rows:
        if int(r["Dispatch_Id"]) < start:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mcrc_dev::", "")
        tot[k] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in calls.items()}


def main():
    first = sys.argv[5] if len(sys.argv) > 5 else "k_census"
    f, fc = per_kernel(sys.argv[1], "FETCH_SIZE", first)
    w, _ = per_kernel(sys.argv[2], "WRITE_SIZE", first)
    batches = max(v for k, v in fc.items() if k.startswith(first))
    algo = float(sys.argv[3])
    rec = {"batches": batches, "batch_starts_at": first, "algorithmic_bytes_per_batch": algo,
           "per_kernel_bytes_per_batch": {}}
    total = 0.0
    for k in sorted(set(f) | set(w)):
        b = (f.get(k, 0) * 2 + w.get(k, 0)) * 1024 / batches
        rec["per_kernel_bytes_per_batch"][k] = b
        total += b
    rec["hbm_bytes_per_batch"] = total
    rec["traffic_over_algorithmic"] = total / algo
    rec["correction"] = "FETCH_SIZE x 2 (gfx950), WRITE_SIZE x 1, KiB -> bytes"
    json.dump(rec, open(sys.argv[4], "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
