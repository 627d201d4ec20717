#!/bin/bash
# Round 5 evidence, part 2: HBM traffic (FETCH_SIZE and WRITE_SIZE in
# separate passes) of the K5 verify (config 5), the stamp and the mixed
# pages, 100 pages each, per batch against the algorithmic bytes.
#   bash tools/r05_traffic.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05tr}; mkdir -p $O
run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
for w in config5 stamp pagesmix; do
  for c in FETCH_SIZE WRITE_SIZE; do
    run 120 rocprofv3 --pmc $c -d $O/${w}_$c -o p --output-format csv -- python3 bench.py --workload $w --pages 100 --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/${w}_$c.log 2>&1
  done
done
echo done
