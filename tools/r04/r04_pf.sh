#!/bin/bash
# Past-the-end prefetch to L2-hot lines (K1, k_lines): A/B and traffic.
#   bash tools/r04_pf.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/k1pf/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "k1 or fixed or golden_all or fuzz or k5 or 4133 or census or async or bench_layout" > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
for r in $(seq 1 $R); do
  for n in base k1pf; do
    echo "== round $r lib $n workload config2" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 50 --warmup 20 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
  for n in k5lines k1pf; do
    for w in config2r config5; do
      case $w in config2r) a="--workload $w --steps 10 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
MCRC_LIB=ab/k1pf/libmcrc32c.so run 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_k1pf_config2 -o f --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch_k1pf_config2.log 2>&1
MCRC_LIB=ab/k1pf/libmcrc32c.so run 90 rocprofv3 --pmc WRITE_SIZE -d $O/write_k1pf_config2 -o w --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/write_k1pf_config2.log 2>&1
for w in config2r config5; do
  a="--workload $w --steps 2 --warmup 1"; [ $w = config5 ] && a="$a --pages 100"
  MCRC_LIB=ab/k1pf/libmcrc32c.so run 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_k1pf_$w -o f --output-format csv -- python3 bench.py $a > $O/fetch_k1pf_$w.log 2>&1
done
echo done
