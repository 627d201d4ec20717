#!/bin/bash
# k_walk variants (abl/libmcrc32c_<name>.so) on the pages workload, rocprofv3 kernel trace
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-walkvar}; mkdir -p $O; shift
for v in base "$@"; do
  lib=$PWD/abl/libmcrc32c_$v.so; [ "$v" = base ] && lib=
  MCRC_LIB=$lib run 300 rocprofv3 --kernel-trace -d $O/$v -o $v --output-format csv -- python3 bench.py --workload pages --pages 300 --steps 3 --warmup 1 > $O/$v.json 2> $O/$v.err
done
echo done
