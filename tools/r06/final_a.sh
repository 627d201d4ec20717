#!/bin/bash
# Round 6 evidence, part A: GPU suite (verbose names), smoke, headline bench
# (driver's arguments), rocprofv3 kernel stats of the headline, K1 HBM traffic
# (FETCH_SIZE / WRITE_SIZE in separate --pmc passes).
#   bash tools/r06/final_a.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r06fin}; mkdir -p $O
run 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py > $O/bench.json 2> $O/bench.err
# the driver's N > 1 launcher, rehearsed at N = 1 (one rank over RCCL)
run 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_torchrun.json 2> $O/bench_torchrun.err
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err
run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch.log 2>&1
run 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/write.log 2>&1
run 60 python tools/traffic.py $O/fetch $O/write $O/traffic.json > /dev/null
echo done
