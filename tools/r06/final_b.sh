#!/bin/bash
# Round 6 evidence, part B: every extra workload once on one box (1000 pages),
# the config-3 / mixed-pages / config-5 kernel traces, the batch_multi call cost.
#   bash tools/r06/final_b.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r06fin}; mkdir -p $O
for w in "config3 --steps 10 --warmup 2" "config2r --steps 10 --warmup 2" "config5 --pages 1000 --steps 5 --warmup 1" \
         "pagesmix --pages 1000 --steps 5 --warmup 1" "pages --pages 1000 --steps 3 --warmup 1" \
         "pagesmixwalk --pages 1000 --steps 3 --warmup 1" "stamp --pages 1000 --steps 3 --warmup 1" \
         "host --steps 5 --warmup 1" "calls" "multi --gpus 1 --steps 20 --warmup 5"; do
  run 600 python bench.py --workload $w --no-cpu-baseline >> $O/extra.jsonl 2>> $O/extra.err
done
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c3 -o c3 --output-format csv -- python3 bench.py --workload config3 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_c3.json 2> $O/kt_c3.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_mix -o mix --output-format csv -- python3 bench.py --workload pagesmix --pages 300 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_mix.json 2> $O/kt_mix.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o c5 --output-format csv -- python3 bench.py --workload config5 --pages 300 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_c5.json 2> $O/kt_c5.err
run 300 python -u tools/r06/multi_overhead.py 500 > $O/multi_overhead.jsonl 2> $O/multi_overhead.err
echo done
