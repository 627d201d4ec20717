"""Per-batch wall time and kernel split of a rocprofv3 --kernel-trace run of a
span workload (config 3, config 5, pages): the library's dispatches grouped
into batches, each batch starting at its first kernel (FIRST), so the batch
time reads directly against bench.py's event-timed kernel_ms.  The rocprof
stats' per-kernel average mixes a batch's large and small dispatches of one
kernel (k_spans: the segment pass and the one-block pass) and the first,
clock-ramping batches; this table does not.
    python tools/ktbatch.py TRACE_CSV FIRST [OUT]"""
import csv
import sys
from collections import defaultdict


def main():
    path, first = sys.argv[1], sys.argv[2]
    rows = [r for r in csv.DictReader(open(path)) if "mcrc_dev" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    batches, cur = [], []
    for r in rows:
        if first in r["Kernel_Name"] and cur:
            batches.append(cur)
            cur = []
        cur.append(r)
    if cur:
        batches.append(cur)
    lines = [f"batches from {path} (a batch starts at {first})",
             "batch  dispatches  wall_ms   sum_ms   kernels (ms, in launch order)"]
    for i, b in enumerate(batches):
        s = min(int(r["Start_Timestamp"]) for r in b)
        e = max(int(r["End_Timestamp"]) for r in b)
        tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in b)
        per = defaultdict(float)
        for r in b:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mcrc_dev::", "")
            per[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        split = ", ".join(f"{k} {v:.4f}" for k, v in per.items())
        lines.append(f"{i:5d}  {len(b):10d}  {(e - s) / 1e6:7.4f}  {tot / 1e6:7.4f}   {split}")
    full = [b for b in batches if len(b) == max(len(x) for x in batches)]
    if len(full) > 2:
        walls = sorted((max(int(r["End_Timestamp"]) for r in b) - min(int(r["Start_Timestamp"]) for r in b)) / 1e6
                       for b in full[2:])
        lines.append(f"complete batches after the first two: wall {walls[0]:.4f}-{walls[-1]:.4f} ms, "
                     f"median {walls[len(walls) // 2]:.4f} ms")
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text + "\n")


if __name__ == "__main__":
    main()
