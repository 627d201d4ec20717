"""HBM traffic per batch of the span workloads (config 3, config 5) from
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (tools/s3_traffic.sh): every
library kernel of the batch, summed per batch (one k_count dispatch per
batch; config 5 with K5: one k_items dispatch per batch), against the
algorithmic bytes.  gfx950 correction as tools/traffic.py
(FETCH_SIZE x 2, KiB).
    python tools/traffic_spans.py FETCH_DIR WRITE_DIR ALGO_BYTES OUT"""
import csv
import glob
import json
import sys
from collections import defaultdict

SETUP = ("k_final<0, false>", "k_spans<false>", "k_blocks<true")  # config 5: the bench's stored CRCs


def per_kernel(d, counter):
    tot, calls = defaultdict(float), defaultdict(set)
    for r in csv.DictReader(open(glob.glob(f"{d}/*counter_collection.csv")[0])):
        n = r["Kernel_Name"]
        if "mcrc" not in n or r["Counter_Name"] != counter or any(s in n for s in SETUP):
            continue
        k = n.split("(")[0].replace("void ", "").replace("mcrc_dev::", "")
        tot[k] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in calls.items()}


f, fc = per_kernel(sys.argv[1], "FETCH_SIZE")
w, _ = per_kernel(sys.argv[2], "WRITE_SIZE")
batches = max(v for k, v in fc.items() if k.startswith(("k_count", "k_items")))
algo = float(sys.argv[3])
rec = {"batches": batches, "algorithmic_bytes_per_batch": algo, "per_kernel_bytes_per_batch": {}}
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
