#!/bin/bash
# Round-4 A/B session on one box: GPU parity of each candidate library (the
# K1/span/item tests), then ROUNDS alternating bench runs of the named
# workloads, then a PMC census (LDS conflicts / instruction counts) per lib.
#   bash tools/r04_ab.sh OUT ROUNDS "lib1 lib2" "workload1 workload2"
#   (lib = a directory under ab/; workloads: config2, config2r, config3, config5, stamp)
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; L=$3; W=$4
mkdir -p $O
for n in $L; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "${TESTS:-k1 or fixed or golden or fuzz or k5 or stamp or 4133 or bench_layout}" \
    > $O/pytest_$n.log 2>&1
  tail -1 $O/pytest_$n.log
done
for r in $(seq 1 $R); do
  for n in $L; do
    for w in $W; do
      case $w in
        config2) a="--steps 50 --warmup 20 --no-cpu-baseline";;
        config5|stamp) a="--workload $w --pages 300 --steps 5 --warmup 1";;
        *) a="--workload $w --steps 10 --warmup 2";;
      esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
if [ -n "$PMC" ]; then
  for n in $L; do
    for w in $W; do
      case $w in config2) a="--steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline";; config5|stamp) a="--workload $w --pages 100 --steps 2 --warmup 1";; *) a="--workload $w --steps 2 --warmup 1";; esac
      MCRC_LIB=ab/$n/libmcrc32c.so run 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${n}_${w}_a -o a --output-format csv -- python3 bench.py $a > $O/pmc_${n}_${w}_a.log 2>&1
      MCRC_LIB=ab/$n/libmcrc32c.so run 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $O/pmc_${n}_${w}_b -o b --output-format csv -- python3 bench.py $a > $O/pmc_${n}_${w}_b.log 2>&1
    done
  done
fi
echo done
