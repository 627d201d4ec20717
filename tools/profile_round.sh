#!/bin/bash
# Round evidence: GPU tests, smoke, headline bench (driver's arguments),
# rocprofv3 kernel stats of the headline, HBM traffic (FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes), span-workload kernel splits.
#   bash tools/profile_round.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-prof}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err
run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch.log 2>&1
run 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/write.log 2>&1
run 60 python tools/traffic.py $O/fetch $O/write $O/traffic.json > /dev/null
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c3 -o c3 --output-format csv -- python3 bench.py --workload config3 --steps 3 --warmup 1 > $O/kt_c3.json 2> $O/kt_c3.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o c5 --output-format csv -- python3 bench.py --workload config5 --pages 300 --steps 3 --warmup 1 > $O/kt_c5.json 2> $O/kt_c5.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2r -o c2r --output-format csv -- python3 bench.py --workload config2r --steps 5 --warmup 1 > $O/kt_c2r.json 2> $O/kt_c2r.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5k -o c5k --output-format csv -- python3 bench.py --workload config5 --pages 1000 --steps 3 --warmup 1 > $O/kt_c5k.json 2> $O/kt_c5k.err
echo done
