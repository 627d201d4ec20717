#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r03e}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
run 300 python bench.py --workload config2r --steps 10 --warmup 2 > $O/config2r.json 2> $O/config2r.err
run 300 python bench.py --workload config5 --pages 1000 --steps 5 --warmup 1 > $O/config5.json 2> $O/config5.err
run 300 python bench.py --workload stamp --pages 1000 --steps 3 --warmup 1 > $O/stamp.json 2> $O/stamp.err
run 300 python bench.py --workload pages --pages 1000 --steps 3 --warmup 1 > $O/pages.json 2> $O/pages.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o c5 --output-format csv -- python3 bench.py --workload config5 --pages 300 --steps 3 --warmup 1 > $O/kt_c5.json 2> $O/kt_c5.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2r -o c2r --output-format csv -- python3 bench.py --workload config2r --steps 5 --warmup 1 > $O/kt_c2r.json 2> $O/kt_c2r.err
echo done
