#!/bin/bash
# The C integration harnesses against an AddressSanitizer build of the
# library's host code (device code unchanged; -Xarch_host only), on the GPU.
#   bash tools/asan_host.sh OUT     (after bash tools/build_asan.sh here)
# (the harnesses are built with ROCm's clang so that they and the library share
# one AddressSanitizer runtime)
source tools/gpu_guard.sh
O=gpurun_out/${1:-asan}; mkdir -p $O
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1
for n in queue_sim extstore_sim storage_sim extstore_config1; do
  /opt/rocm/lib/llvm/bin/clang -O1 -g -fsanitize=address -fno-omit-frame-pointer -pthread -I include tests/integration/$n.c \
      -L ab -lmcrc32c_asan -Wl,-rpath,$PWD/ab -o /tmp/asan_$n || exit 1
done
run 120 /tmp/asan_queue_sim --gpu 16 500 1 > $O/queue_16x1.txt 2>&1
run 120 /tmp/asan_queue_sim --gpu 8 200 8 > $O/queue_8x8.txt 2>&1
run 120 /tmp/asan_extstore_sim --gpu 8 > $O/extstore.txt 2>&1
run 120 /tmp/asan_storage_sim --gpu > $O/storage.txt 2>&1
mkdir -p /tmp/asan_c1 && run 120 /tmp/asan_extstore_config1 /tmp/asan_c1 --gpu > $O/config1.txt 2>&1
grep -l "ERROR: AddressSanitizer" $O/*.txt > $O/asan_errors.txt || echo "no AddressSanitizer reports" > $O/asan_errors.txt
echo done
