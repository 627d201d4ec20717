#!/bin/bash
# AddressSanitizer build of the library's host code (the device code is
# compiled as usual: -fsanitize only after -Xarch_host) into ab/, for
# tools/asan_host.sh.  Runs here (no GPU needed).
set -e
H=/opt/rocm/bin/hipcc
mkdir -p ab
$H --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer \
   -c memcached_amd/csrc/crc32c_shim.hip -o /tmp/shim_asan.o
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fPIC -fsanitize=address -fno-omit-frame-pointer \
   -c memcached_amd/csrc/crc32c_host.cpp -o /tmp/host_asan.o
$H --offload-arch=gfx950 -shared -fPIC -fsanitize=address -o ab/libmcrc32c_asan.so /tmp/shim_asan.o /tmp/host_asan.o -lpthread
echo ab/libmcrc32c_asan.so
