#!/bin/bash
# One GPU-box session: smoke, GPU tests, bench, rocprofv3 kernel-trace summaries
# of the bench and of every profiled pass, and the PMC passes (traffic and VALU /
# MFMA issue counters) per pass.  Every GPU step has its own time limit; a
# fault / abort / timeout ends the script (exit codes other than 0, 1).
# Usage: bash tools/gpu_check.sh [tag] [quick]
set -u
TAG=${1:-r03}
QUICK=${2:-}
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
TAILN=12 CNF_RECORD_DIR=gpurun_out run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
TAILN=2 run bench 600 python bench.py
[ -n "$QUICK" ] && exit 0
run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 200 --no-cpu-baseline --no-variants
# the bench's own timed steps: its last 200 + 100 calls (the timed region and
# the kernel-only pass, both after the settle and the warmup)
python tools/trace_stats.py gpurun_out/prof_$TAG/run_kernel_trace.csv 300 gpurun_out/prof_$TAG/settled_stats.csv
# one kernel-trace summary per profiled pass, the clock settled first (0.3 s,
# as bench.py), statistics over the last N calls only (tools/trace_stats.py)
for spec in "cfg2 loss 200 k_sgpr" "cfg2 forward 200 k_sgpr" "cfg2 all 100 k_valu" "cfg5 forward 200 k_sgpr" "cfg4 forward 10 k_wide16" "cfg2 train 100 k_vjp2" "cfg4 train 5 k_wtrain16_fwd"; do
  set -- $spec
  run rocprof_$1_$2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$1_$2 -o run --output-format csv -- python tools/prof_target.py --workload $1 --mode $2 --launches $3
  python tools/trace_stats.py gpurun_out/prof_${TAG}_$1_$2/run_kernel_trace.csv $3 gpurun_out/prof_${TAG}_$1_$2/settled_stats.csv $4
done
run sweep_loss 300 python tools/batch_sweep.py loss
run sweep_fwd 300 python tools/batch_sweep.py forward
# PMC passes: HBM traffic (separate FETCH / WRITE passes) and issue counters
VALU="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
MFMA="SQ_WAVES SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for spec in "cfg2 loss k_sgpr" "cfg2 all k_valu" "cfg2 train k_vjp2" "cfg4 forward k_wide16" "cfg4 train k_wdw16"; do
  set -- $spec
  rm -rf gpurun_out/pmc_${TAG}_$1_$2_$1
  CTR="$VALU"; case "$3" in k_wide*|k_vjp2|k_wdw*) CTR="$MFMA";; esac
  NL=20; [ "$1 $2" = "cfg4 train" ] && NL=2
  run pmc_$1_$2 600 bash tools/gpu_pmc.sh ${TAG}_$1_$2 $1 "--mode $2 --launches $NL --settle-s 0" "FETCH_SIZE" "WRITE_SIZE" "$CTR"
  python tools/pmc_summary.py gpurun_out/pmc_${TAG}_$1_$2_$1 $3 > gpurun_out/${TAG}_pmc_$1_$2.txt 2>&1
done
# the fused wide training sweeps, from the cfg4 train pass
for k in k_wtrain16_fwd k_wtrain16_bwd; do
  python tools/pmc_summary.py gpurun_out/pmc_${TAG}_cfg4_train_cfg4 $k > gpurun_out/${TAG}_pmc_cfg4_train_$k.txt 2>&1
done
exit 0
