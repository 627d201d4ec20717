#!/bin/bash
# Build ablation variants of the library (run in the build container):
#   tools/ablate_spans.sh build NAME -DFLAG ...   -> gpurun_abl/libmcrc32c_NAME.so
# and time them on the GPU box:
#   tools/ablate_spans.sh run OUT NAME...
set -e
if [ "$1" = build ]; then
    name=$2; shift 2
    mkdir -p abl
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c memcached_amd/csrc/crc32c_shim.hip -o abl/$name.o
    g++ -O2 -std=c++17 -fPIC -c memcached_amd/csrc/crc32c_host.cpp -o abl/host.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libmcrc32c_$name.so abl/$name.o abl/host.o -lpthread
    rm -f abl/*.o
    exit 0
fi
source tools/gpu_guard.sh
O=gpurun_out/$2; mkdir -p $O; shift 2
for v in "$@"; do
    lib=$PWD/abl/libmcrc32c_$v.so; [ "$v" = base ] && lib=
    MCRC_LIB=$lib run 300 python bench.py --no-cpu-baseline --steps 30 > $O/c2_$v.json 2> $O/c2_$v.err
    MCRC_LIB=$lib run 300 python bench.py --workload config2r --steps 10 --warmup 2 > $O/c2r_$v.json 2> $O/c2r_$v.err
    MCRC_LIB=$lib run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 1 > $O/c5_$v.json 2> $O/c5_$v.err
    MCRC_LIB=$lib run 300 python bench.py --workload config3 --steps 5 --warmup 1 > $O/c3_$v.json 2> $O/c3_$v.err
done
echo done
