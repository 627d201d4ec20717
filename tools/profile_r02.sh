#!/bin/bash
# Round-2 evidence: GPU tests, smoke, headline bench (driver's arguments and
# defaults), rocprofv3 kernel stats of the headline, HBM traffic (separate
# --pmc passes), span workload kernel splits and extra workload lines.
#   bash tools/profile_r02.sh r02
source tools/gpu_guard.sh
export TMPDIR=/tmp
R=${1:-r02}
O=gpurun_out/$R; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
run 300 python bench.py > $O/bench_default.json 2>> $O/bench.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err
run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch.log 2>&1
run 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/write.log 2>&1
run 60 python tools/traffic.py $O/fetch $O/write $O/traffic.json > /dev/null
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c3 -o c3 --output-format csv -- python3 bench.py --workload config3 --steps 3 --warmup 1 > $O/kt_c3.json 2> $O/kt_c3.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o c5 --output-format csv -- python3 bench.py --workload config5 --pages 300 --steps 3 --warmup 1 > $O/kt_c5.json 2> $O/kt_c5.err
echo done
# (extra workload lines: bash tools/extra_workloads.sh $R/x, a call of its own)
