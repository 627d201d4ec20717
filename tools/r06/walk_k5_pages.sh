source tools/gpu_guard.sh
O=gpurun_out/r06_wk5q; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for p in 1024 1000; do for m in 0 2; do
  run 300 rocprofv3 --kernel-trace --stats -d $O/p${p}m$m -o k --output-format csv -- python bench.py --workload pages --walk-mode $m --pages $p --steps 5 --no-cpu-baseline > $O/p${p}m$m.json 2> $O/p${p}m$m.err
done; done
echo done
