#!/bin/bash
# Round-4 evidence, part 2: the page workloads (1000 x 64 MiB pages) and the
# per-call / multi / host workloads, with kernel traces.
#   bash tools/r04_final2.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r04final2}; mkdir -p $O
for w in config5 stamp pages pagesmix; do
  a="--workload $w --pages 1000 --steps 3 --warmup 1"
  run 600 python bench.py $a > $O/$w.json 2> $O/$w.err
  run 600 rocprofv3 --kernel-trace --stats -d $O/kt_$w -o kt --output-format csv -- python3 bench.py --workload $w --pages 300 --steps 3 --warmup 1 > $O/kt_$w.json 2> $O/kt_$w.err
done
for w in config3 config2r; do
  case $w in config3) a="--workload $w --steps 5 --warmup 2";; *) a="--workload $w --steps 10 --warmup 2";; esac
  run 600 python bench.py $a > $O/$w.json 2> $O/$w.err
done
run 600 rocprofv3 --kernel-trace --stats -d $O/kt_config3 -o kt --output-format csv -- python3 bench.py --workload config3 --steps 5 --warmup 2 > $O/kt_config3.json 2> $O/kt_config3.err
run 300 python bench.py --workload calls > $O/calls.json 2> $O/calls.err
run 300 python bench.py --workload multi --gpus 1 --steps 20 --warmup 5 > $O/multi.json 2> $O/multi.err
run 300 python bench.py --workload host --steps 5 --warmup 1 > $O/host.json 2> $O/host.err
for w in config2r config5; do
  a="--workload $w --steps 2 --warmup 1"; [ $w = config5 ] && a="$a --pages 100"
  run 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$w -o f --output-format csv -- python3 bench.py $a > $O/fetch_$w.log 2>&1
done
echo done
