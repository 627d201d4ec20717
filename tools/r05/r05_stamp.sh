#!/bin/bash
# Round 5, review item 1: where the spill stamp's time goes.  Same box, one
# session: the stamp (k_census + k_lines<2> + k_fix + fallback) under each
# store variant of ab/NAME (tools/ab_lib.sh; the variants are compile-time
# switches of a scratch build), beside the verify over identical pages.
#   cur     4 non-temporal byte stores per image in k_fix (the round-4 build)
#   fixdw   one non-temporal dword store (unaligned) in k_fix
#   fixdwp  one plain dword store in k_fix
#   fix32nt the 32-B sector(s) holding exptime re-written whole (NT)
#   fix32   the same with plain stores
#   nofix   no k_fix (timing only: no stamps written)
#   lnst    k_lines<2>'s epoch lane stores the CRC (NT dword), no k_fix
#   lnnort  k_lines<2> without its {V, pad} store and no k_fix (timing only)
#   bash tools/r05_stamp.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
for n in fixdw fix32nt lnst; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "stamp or extstore or config1" > $O/pytest_$n.log 2>&1
  tail -1 $O/pytest_$n.log
done
for r in $(seq 1 $R); do
  for n in cur fixdw fixdwp fix32nt fix32 nofix lnst lnnort; do
    echo "== round $r lib $n workload stamp" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload stamp --pages 300 --steps 5 --warmup 1 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
  echo "== round $r lib cur workload config5" >> $O/ab.txt
  MCRC_LIB=ab/cur/libmcrc32c.so run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 1 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
done
echo done
