#!/bin/bash
# k_lines stamps stored by the epoch lanes (stamp) against {V, pad} + k_fix
# (cur): stamp parity with the stamp build, A/B, fetch and write traffic;
# the page walk's emit pass copying the count pass's offsets (walk1) against
# walking every wbuf twice (cur).
#   bash tools/r04_stamp.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/stamp/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "k5 or census or async or stamp or items or pages or config1 or extstore" > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur stamp; do
    for w in stamp config5; do
      a="--workload $w --pages 300 --steps 5 --warmup 1"
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
MCRC_LIB=ab/walk1/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "walk or pages or k5" > $O/pytest_gpu_walk1.log 2>&1
tail -1 $O/pytest_gpu_walk1.log
grep -q " passed" $O/pytest_gpu_walk1.log && ! grep -q "failed" $O/pytest_gpu_walk1.log || { echo "walk tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur walk1; do
    echo "== round $r lib $n workload pages" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload pages --pages 300 --steps 5 --warmup 1 >> $O/ab.txt 2>> $O/ab.err
  done
done
for n in cur stamp; do
  for c in FETCH_SIZE WRITE_SIZE; do
    MCRC_LIB=ab/$n/libmcrc32c.so run 120 rocprofv3 --pmc $c -d $O/pmc_${n}_$c -o p --output-format csv -- python3 bench.py --workload stamp --pages 100 --steps 2 --warmup 1 --settle-ms 0 > $O/pmc_${n}_$c.log 2>&1
  done
done
bash tools/r04_cnt.sh $1 3 || exit 1
MCRC_LIB=ab/walk1/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_config2r -o kt --output-format csv -- python3 bench.py --workload config2r --steps 20 --warmup 2 > $O/kt_config2r.json 2> $O/kt_config2r.err
echo all done
