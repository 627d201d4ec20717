#!/bin/bash
# Round 5: every table kernel on K1's coalesced non-temporal pieces (k_spans,
# k_small, k_blocks, k_lines) and one chunk-16 table image.  Full GPU parity,
# smoke, then an interleaved A/B against the previous build (ab/head: K1 and
# k_lines converted, the span kernels not; ab/pieces: this build) on the
# planned-path workloads and K5's.
#   bash tools/r05_spans.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05sp}; R=${2:-2}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed, stopping"; exit 1; }
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in $(seq 1 $R); do
  for n in head pieces; do
    for w in "config3" "pagesmix --pages 300" "config5 --pages 300" "pages --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
