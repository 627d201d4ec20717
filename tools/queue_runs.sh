#!/bin/bash
# Coalescing-queue measurements: queue_sim (tests/integration) at several
# thread counts and IO-batch depths; one summary line per run.
#   bash tools/queue_runs.sh OUTFILE
source tools/gpu_guard.sh
OUT=${1:-gpurun_out/queue.txt}
mkdir -p "$(dirname "$OUT")"
EXE=/tmp/queue_sim_$$
gcc -O2 -pthread -I include tests/integration/queue_sim.c -L memcached_amd -lmcrc32c \
    -Wl,-rpath,"$PWD/memcached_amd" -o $EXE || exit 1
: > "$OUT"
for cfg in "1 3000 1" "4 3000 1" "16 3000 1" "64 1500 1" "128 800 1" "16 1500 8" "64 500 8" "64 200 64"; do
    run 120 $EXE --gpu $cfg >> "$OUT" 2>&1
done
rm -f $EXE
