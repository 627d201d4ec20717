#!/bin/bash
source tools/gpu_guard.sh
O=gpurun_out/${1:-x1}; mkdir -p $O
run 600 python bench.py --workload config3 --steps 10 --warmup 2 > $O/config3.json 2> $O/config3.err
run 600 python bench.py --workload config5 --pages ${PAGES:-1000} --steps 5 --warmup 1 > $O/config5.json 2> $O/config5.err
run 600 python bench.py --workload config2r --steps 10 --warmup 2 > $O/config2r.json 2> $O/config2r.err
run 600 python bench.py --workload pagesmix --pages ${PAGES:-1000} --steps 5 --warmup 1 > $O/pagesmix.json 2> $O/pagesmix.err
run 600 python bench.py --workload pages --pages ${PAGES:-1000} --steps 3 --warmup 1 > $O/pages.json 2> $O/pages.err
run 600 python bench.py --workload stamp --pages ${PAGES:-1000} --steps 3 --warmup 1 > $O/stamp.json 2> $O/stamp.err
run 600 python bench.py --workload host --steps 5 --warmup 1 > $O/host.json 2> $O/host.err
run 600 python bench.py --workload calls > $O/calls.json 2> $O/calls.err
echo done
