#!/bin/bash
# activity counters of the pipelined-scalar kernel at 1M and 8M (forward)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 1048576 8388608; do
  bash tools/gpu_pmc.sh sg$B cfg2 "--launches 20 --mode forward --batch $B" \
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
    "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
    "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM" \
    "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU" || exit $?
done
exit 0
