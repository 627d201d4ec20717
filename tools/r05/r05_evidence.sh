#!/bin/bash
# Round 5 evidence, part 1: every workload at its full size on one box
# (1000 pages), the per-batch kernel traces of the span workloads.
#   bash tools/r05_evidence.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ev}; mkdir -p $O
run 600 python bench.py --workload config3 --steps 10 --warmup 2 > $O/config3.json 2> $O/config3.err
run 600 python bench.py --workload config5 --pages 1000 --steps 5 --warmup 1 > $O/config5.json 2> $O/config5.err
run 600 python bench.py --workload config2r --steps 10 --warmup 2 > $O/config2r.json 2> $O/config2r.err
run 600 python bench.py --workload pagesmix --pages 1000 --steps 5 --warmup 1 > $O/pagesmix.json 2> $O/pagesmix.err
run 600 python bench.py --workload pages --pages 1000 --steps 3 --warmup 1 > $O/pages.json 2> $O/pages.err
run 600 python bench.py --workload stamp --pages 1000 --steps 3 --warmup 1 > $O/stamp.json 2> $O/stamp.err
run 600 python bench.py --workload host --steps 5 --warmup 1 > $O/host.json 2> $O/host.err
run 300 python bench.py --workload multi --gpus 1 --steps 20 --warmup 5 > $O/multi.json 2> $O/multi.err
for w in "config5 --pages 300" "stamp --pages 300" "pagesmix --pages 300" "config2r" "config3"; do
  n=$(echo $w | cut -d' ' -f1)
  run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_$n.json 2> $O/kt_$n.err
done
echo done
