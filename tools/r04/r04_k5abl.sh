#!/bin/bash
# K5 ablations (wrong results, timing only): where config 2r loses against K1.
#   bash tools/r04_k5abl.sh OUT ROUNDS "libs"
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; L=$3; mkdir -p $O
for r in $(seq 1 $R); do
  for n in $L; do
    echo "== round $r lib $n workload config2r" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload config2r --steps 10 --warmup 2 >> $O/ab.txt 2>> $O/ab.err
    echo "== round $r lib $n workload config5" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 1 >> $O/ab.txt 2>> $O/ab.err
  done
done
for n in $L; do
  for w in config2r config5; do
    a="--workload $w --steps 2 --warmup 1"; [ $w = config5 ] && a="$a --pages 100"
    MCRC_LIB=ab/$n/libmcrc32c.so run 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_${n}_$w -o f --output-format csv -- python3 bench.py $a > $O/fetch_${n}_$w.log 2>&1
  done
done
echo done
