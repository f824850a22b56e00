#!/bin/bash
# One GPU-box session: smoke, GPU tests, bench, rocprofv3 kernel-trace summary,
# and the PMC traffic passes for the bench kernel.  Every GPU step has its own
# time limit; a fault/abort/timeout ends the script (exit codes other than 0, 1).
# Usage: bash tools/gpu_check.sh [tag]
set -u
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  local t0=$(date +%s)
  timeout -k 10 "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc ($(( $(date +%s) - t0 ))s)"
  tail -n ${TAILN:-5} gpurun_out/$name.log | grep -v amdgpu.ids
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -m pytest tests -m gpu -q
TAILN=2 run bench 600 python bench.py
run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 100 --no-cpu-baseline --no-variants
rm -rf gpurun_out/pmc_${TAG}_cfg2
run pmc 600 bash tools/gpu_pmc.sh $TAG cfg2 "--launches 30" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
python tools/pmc_traffic.py gpurun_out/pmc_${TAG}_cfg2 gpurun_out/${TAG}_traffic_cfg2.json cfg2 1048576 k_sgpr > /dev/null && cat gpurun_out/${TAG}_traffic_cfg2.json
exit 0
