#!/bin/bash
# One iteration: GPU tests (stop on failure), then VALU census + timings of
# cur vs the given libraries on config2r / config3 / config5.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "$@"; do
  lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
  for w in config2r config3; do
    MCRC_LIB=$lib run 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/${v}-${w}_a -o a --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 > $O/${v}-${w}_a.log 2>&1
  done
done
for i in 1 2; do for v in "$@"; do
  lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
  MCRC_LIB=$lib run 120 python bench.py --workload config2r --steps 10 --warmup 3 > $O/${v}-c2r_$i.json 2>>$O/err.log
  MCRC_LIB=$lib run 120 python bench.py --workload config3 --steps 5 --warmup 2 > $O/${v}-c3_$i.json 2>>$O/err.log
  MCRC_LIB=$lib run 120 python bench.py --workload config5 --pages 300 --steps 5 --warmup 2 > $O/${v}-c5_$i.json 2>>$O/err.log
done; done
echo done
