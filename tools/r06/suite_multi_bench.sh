#!/bin/bash
# Round 6: the full GPU suite + smoke, the batch_multi per-call cost at N = 1,
# and one default bench line.
#   bash tools/r06/suite_multi_bench.sh OUT
source tools/gpu_guard.sh
O=${1:-r06b}
mkdir -p gpurun_out/$O
bash tools/gpu_suite.sh $O/suite || exit $?
run 300 python -u tools/r06/multi_overhead.py 500 > gpurun_out/$O/multi_overhead.jsonl 2> gpurun_out/$O/multi_overhead.err
run 300 python -u bench.py > gpurun_out/$O/bench.json 2> gpurun_out/$O/bench.err
