#!/bin/bash
# Round 6, first GPU call: the 64-bit shift / top-VGPR experiment, then the
# full GPU suite and smoke on the alignbyte parse_hdr.
#   bash tools/r06/shift_and_suite.sh OUT
source tools/gpu_guard.sh
O=${1:-r06a}
bash tools/shift64_top_vgpr.sh $O/shift64 300 || exit $?
bash tools/gpu_suite.sh $O/suite
