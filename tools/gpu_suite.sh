#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05suite}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo done
