#!/bin/bash
# Round 6: k_fix with a per-workgroup table of x^(-8 (t + 128)) (cur) against
# two multiplies per image (HEAD): stamp GPU tests on cur, stamp A/B.
#   bash tools/r06/kfix_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_kfix}; R=${2:-3}
mkdir -p $O
run 600 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "stamp or k5 or lines or integration or planned_rounds" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for r in $(seq 1 $R); do
  for n in HEAD cur; do
    echo "== round $r lib $n workload stamp" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload stamp --pages 1000 --steps 3 --warmup 1 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --workload stamp --pages 300 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt.json 2> $O/kt.err
echo done
