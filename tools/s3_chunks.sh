#!/bin/bash
# Chunked plans: GPU tests, then config 5 / stamp A/B against the single-pass plan.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3ch}; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2 3; do
  for v in cur single; do
    e=; [ $v = single ] && e=1
    MCRC_NO_CHUNKS=$e run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 2 > $O/${v}_c5_$i.json 2>>$O/err.log
    MCRC_NO_CHUNKS=$e run 300 python bench.py --workload stamp --pages 300 --steps 5 --warmup 2 > $O/${v}_stamp_$i.json 2>>$O/err.log
  done
done
run 200 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o kt --output-format csv -- python3 bench.py --workload config5 --steps 3 --warmup 1 --pages 300 > $O/kt_c5.log 2>&1
echo done
