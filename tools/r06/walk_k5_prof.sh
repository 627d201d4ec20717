#!/bin/bash
# Round 6: kernel traces of crc32c_verify_pages on config 5's pages by walk
# mode (0 two-pass, 1 default, 2 one-pass forced) and of config 5's item list.
#   bash tools/r06/walk_k5_prof.sh OUT
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_wk5p}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in 0 1 2; do
  run 300 rocprofv3 --kernel-trace --stats -d $O/m$m -o m$m --output-format csv -- python bench.py --workload pages --walk-mode $m --pages 1000 --steps 5 --no-cpu-baseline > $O/m$m.json 2> $O/m$m.err
done
run 300 rocprofv3 --kernel-trace --stats -d $O/c5 -o c5 --output-format csv -- python bench.py --workload config5 --pages 1000 --steps 5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
echo done
