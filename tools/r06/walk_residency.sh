source tools/gpu_guard.sh
O=gpurun_out/r06_mix500; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for p in 500 1000 250; do
  run 300 rocprofv3 --kernel-trace --stats -d $O/p$p -o k --output-format csv -- python bench.py --workload pagesmixwalk --pages $p --steps 3 --no-cpu-baseline > $O/p$p.json 2> $O/p$p.err
done
echo done
