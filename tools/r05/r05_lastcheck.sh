#!/bin/bash
# Round 5, last GPU check of the committed build on a fresh box: GPU suite,
# smoke, headline, and the span workloads at full size (no profiler).
#   bash tools/r05_lastcheck.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05last}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed, stopping"; exit 1; }
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
run 600 python bench.py --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > $O/config3.json 2> $O/config3.err
run 600 python bench.py --workload pagesmix --pages 1000 --steps 5 --warmup 1 --no-cpu-baseline > $O/pagesmix.json 2> $O/pagesmix.err
run 600 python bench.py --workload config5 --pages 1000 --steps 5 --warmup 1 --no-cpu-baseline > $O/config5.json 2> $O/config5.err
run 600 python bench.py --workload stamp --pages 1000 --steps 3 --warmup 1 --no-cpu-baseline > $O/stamp.json 2> $O/stamp.err
run 600 python bench.py --workload config2r --steps 10 --warmup 2 --no-cpu-baseline > $O/config2r.json 2> $O/config2r.err
echo done
