#!/bin/bash
# Round 6: what bounds the walk's count pass -- HBM requests of k_walk<false>
# on config 5's pages (300 pages, two-pass walk), and the counter list.
#   bash tools/r06/count_pass_pmc.sh OUT
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_cpmc}
mkdir -p $O
run 300 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "count_only_query" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run 120 rocprofv3 -L > $O/counters.txt 2>&1
for c in FETCH_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  run 120 rocprofv3 --pmc $c -d $O/$n -o $n --output-format csv -- python bench.py --workload pages --pages 300 --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/$n.log 2>&1
done
echo done
