#!/bin/bash
# Round 5: the coalesced non-temporal K1 -- GPU parity, smoke, headline bench,
# kernel trace, HBM traffic (FETCH_SIZE / WRITE_SIZE passes), the FETCH_SIZE
# correction checked on the microbench's known-byte NT streams, and the
# ceiling microbench on the same box.
#   bash tools/r05_k1.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k1}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err
run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch.log 2>&1
run 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/write.log 2>&1
run 60 python tools/traffic.py $O/fetch $O/write $O/traffic.json > /dev/null
run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_ub -o fub --output-format csv -- tools/k1_ceiling 1 > $O/fetch_ub.log 2>&1
run 300 tools/k1_ceiling 30 > $O/k1_ceiling.txt 2>&1
run 300 python bench.py --workload calls > $O/calls.json 2> $O/calls.err
echo done
