#!/bin/bash
# Round-4 evidence on one box: GPU parity (every test), smoke, the headline
# with the driver's arguments, rocprofv3 kernel stats of the headline and of
# every span workload, HBM traffic of K1 (separate FETCH_SIZE / WRITE_SIZE
# passes) and of k_lines, and the extra workloads' JSON lines.
#   bash tools/r04_final.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r04final}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cat $O/bench.json
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err
run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch.log 2>&1
run 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/write.log 2>&1
run 60 python tools/traffic.py $O/fetch $O/write $O/traffic.json > /dev/null
for w in config3 config2r; do
  case $w in config3) a="--workload $w --steps 5 --warmup 2";; *) a="--workload $w --steps 10 --warmup 2";; esac
  run 600 python bench.py $a > $O/$w.json 2> $O/$w.err
  run 600 rocprofv3 --kernel-trace --stats -d $O/kt_$w -o kt --output-format csv -- python3 bench.py $a > $O/kt_$w.json 2> $O/kt_$w.err
done
echo done
