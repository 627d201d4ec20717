#!/bin/bash
# ThreadSanitizer build of the library's host code into ab/ (tools/tsan_host.sh).
set -e
H=/opt/rocm/bin/hipcc
mkdir -p ab
$H --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Xarch_host -fsanitize=thread -c memcached_amd/csrc/crc32c_shim.hip \
   -o /tmp/shim_tsan.o 2>/dev/null
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fPIC -fsanitize=thread -c memcached_amd/csrc/crc32c_host.cpp \
   -o /tmp/host_tsan.o
$H --offload-arch=gfx950 -shared -fPIC -fsanitize=thread -o ab/libmcrc32c_tsan.so /tmp/shim_tsan.o /tmp/host_tsan.o -lpthread
echo ab/libmcrc32c_tsan.so
