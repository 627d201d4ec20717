#!/bin/bash
# Build a variant of libmcrc32c.so with extra compiler flags into ab/NAME/
# (for A/B runs: MCRC_LIB=ab/NAME/libmcrc32c.so python bench.py ...).
#   bash tools/ab_lib.sh NAME [-DFLAG ...]
set -e
N=$1; shift
mkdir -p ab/$N
g++ -O2 -std=c++17 -fPIC -c memcached_amd/csrc/crc32c_host.cpp -o ab/$N/host.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c memcached_amd/csrc/crc32c_shim.hip -o ab/$N/shim.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/$N/libmcrc32c.so ab/$N/shim.o ab/$N/host.o -lpthread
rm -f ab/$N/*.o
