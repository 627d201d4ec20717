#!/bin/bash
# The threaded C harnesses (coalescing queue, extstore fence) against a
# ThreadSanitizer build of the library's host code (-Xarch_host; the HIP
# runtime itself is not instrumented), on the GPU.
#   bash tools/tsan_host.sh OUT     (after bash tools/build_tsan.sh here)
source tools/gpu_guard.sh
O=gpurun_out/${1:-tsan}; mkdir -p $O
export TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 suppressions=$PWD/tools/tsan_hip.supp"
for n in queue_sim extstore_sim; do
  /opt/rocm/lib/llvm/bin/clang -O1 -g -fsanitize=thread -pthread -I include tests/integration/$n.c \
      -L ab -lmcrc32c_tsan -Wl,-rpath,$PWD/ab -o /tmp/tsan_$n || exit 1
done
run 300 /tmp/tsan_queue_sim --gpu 16 300 1 > $O/queue_16x1.txt 2>&1
run 300 /tmp/tsan_queue_sim --gpu 8 100 8 > $O/queue_8x8.txt 2>&1
run 300 /tmp/tsan_extstore_sim --gpu 8 > $O/extstore.txt 2>&1
grep -c "WARNING: ThreadSanitizer" $O/*.txt > $O/tsan_counts.txt || true
echo done
