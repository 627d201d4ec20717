source tools/gpu_guard.sh
mkdir -p gpurun_out/r04_last
run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_last/pytest_gpu.log 2>&1
tail -1 gpurun_out/r04_last/pytest_gpu.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_last/smoke.log 2>&1
tail -1 gpurun_out/r04_last/smoke.log
run 300 python bench.py > gpurun_out/r04_last/bench.json 2> gpurun_out/r04_last/bench.err
cut -c1-200 gpurun_out/r04_last/bench.json
