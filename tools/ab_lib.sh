#!/bin/bash
# span workloads with the previous library (abl/libmcrc32c_prev.so) vs the
# current one, alternating on one box
source tools/gpu_guard.sh
O=gpurun_out/${1:-ablib}; mkdir -p $O
for i in 1 2; do
  for w in config2r config3; do
    MCRC_LIB=$PWD/abl/libmcrc32c_prev.so run 300 python bench.py --workload $w --steps 10 --warmup 3 > $O/prev_${w}_$i.json 2>/dev/null
    run 300 python bench.py --workload $w --steps 10 --warmup 3 > $O/cur_${w}_$i.json 2>/dev/null
  done
  MCRC_LIB=$PWD/abl/libmcrc32c_prev.so run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 2 > $O/prev_config5_$i.json 2>/dev/null
  run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 2 > $O/cur_config5_$i.json 2>/dev/null
done
echo done
