#!/bin/bash
# Round 5, build evidence: GPU suite, smoke, headline (driver's arguments),
# rocprof stats of the headline, K1 PMC census, the span workloads at full
# size with per-batch traces, traffic of config 3 and the mixed pages.
#   bash tools/r05_final.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05fin}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed, stopping"; exit 1; }
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err
run 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/k1pmc_a -o a --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/k1pmc_a.log 2>&1
run 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $O/k1pmc_b -o b --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/k1pmc_b.log 2>&1
run 600 python bench.py --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > $O/config3.json 2> $O/config3.err
run 600 python bench.py --workload pagesmix --pages 1000 --steps 5 --warmup 1 --no-cpu-baseline > $O/pagesmix.json 2> $O/pagesmix.err
run 600 python bench.py --workload config5 --pages 1000 --steps 5 --warmup 1 --no-cpu-baseline > $O/config5.json 2> $O/config5.err
run 600 python bench.py --workload stamp --pages 1000 --steps 3 --warmup 1 --no-cpu-baseline > $O/stamp.json 2> $O/stamp.err
run 600 python bench.py --workload config2r --steps 10 --warmup 2 --no-cpu-baseline > $O/config2r.json 2> $O/config2r.err
run 600 python bench.py --workload pages --pages 1000 --steps 3 --warmup 1 --no-cpu-baseline > $O/pages.json 2> $O/pages.err
for w in "config3" "pagesmix --pages 300"; do
  n=$(echo $w | cut -d' ' -f1)
  run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_$n.json 2> $O/kt_$n.err
  for c in FETCH_SIZE WRITE_SIZE; do
    run 120 rocprofv3 --pmc $c -d $O/tr_${n}_$c -o p --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/tr_${n}_$c.log 2>&1
  done
done
echo done
