#!/bin/bash
# k_expand one span per thread + big spans from 4 segments: parity and the
# planned path's kernel times (config 3, the K5 fallback of config 5, mixed pages).
#   bash tools/r04_expand.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed, stopping"; exit 1; }
for w in config3 config5 pagesmix config2r; do
  case $w in config3) a="--workload $w --steps 5 --warmup 2";; config2r) a="--workload $w --steps 10 --warmup 2";; *) a="--workload $w --pages 300 --steps 3 --warmup 1";; esac
  run 600 python bench.py $a > $O/$w.json 2> $O/$w.err
  run 600 rocprofv3 --kernel-trace --stats -d $O/kt_$w -o kt --output-format csv -- python3 bench.py $a > $O/kt_$w.json 2> $O/kt_$w.err
done
echo done
