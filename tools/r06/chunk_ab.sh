#!/bin/bash
# Round 6: K5 runs dealt per 16-run chunk (chunk16) against one run at a time
# (cur): config 5 verify at 1000 pages, the K5 tests on chunk16 first.
#   bash tools/r06/chunk_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_chunk}; R=${2:-3}
mkdir -p $O
MCRC_LIB=ab/chunk16/libmcrc32c.so run 300 python -u -m pytest tests/test_gpu_items_queue.py tests/test_gpu_parity.py -q -m gpu \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "k5 or bench_layout or stamp" > $O/pytest_chunk16.log 2>&1
tail -1 $O/pytest_chunk16.log
for r in $(seq 1 $R); do
  for n in cur chunk16; do
    echo "== round $r lib $n" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload config5 --pages 1000 --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
echo done
