#!/bin/bash
# k_lines staggered first runs (stag) against equal runs (nostag); plan tiles
# of 1024 x 2 spans (both builds); config 3 for the plan kernels.
#   bash tools/r04_stag.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/stag/libmcrc32c.so run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in nostag stag; do
    for w in config2r config5; do
      case $w in config2r) a="--workload $w --steps 10 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
MCRC_LIB=ab/stag/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_config3 -o kt --output-format csv -- python3 bench.py --workload config3 --steps 5 --warmup 2 > $O/kt_config3.json 2> $O/kt_config3.err
echo done
