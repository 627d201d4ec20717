#!/bin/bash
# k_lines: per-wave contiguous chunks with staggered runs (chunk) against
# round-robin runs (cur): K5 parity with the chunk build, then A/B.
#   bash tools/r04_chunk.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/chunk/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "k5 or 4133 or census or async or bench_layout or stamp or verify or pages or items" > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur chunk; do
    for w in config2r config5 stamp; do
      case $w in config2r) a="--workload $w --steps 10 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
MCRC_LIB=ab/chunk/libmcrc32c.so run 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_chunk_config2r -o f --output-format csv -- python3 bench.py --workload config2r --steps 2 --warmup 1 > $O/fetch_chunk_config2r.log 2>&1
echo done
