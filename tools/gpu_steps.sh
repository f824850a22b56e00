#!/bin/bash
# Named GPU steps for one gpurun call, each under its own time limit; the first
# step that faults, aborts or times out ends the script (exit codes other than
# 0 / 1, which only mean "tests failed").  Logs: gpurun_out/<step>.log.
# Usage: bash tools/gpu_steps.sh step [step ...]
#   tests        pytest -m gpu (whole GPU suite)
#   smoke        __graft_entry__.smoke()
#   bench        python bench.py (default line)
#   trace        k_sgpr per-wave timeline (libcnf_hip_trace.so), loss + forward
#   rate         tools/quick_rate.py loss / forward (2^20 and 2^23 rows)
#   ab           tools/quick_rate.py $AB_MODE for every tools/ab/lib*.so (make ab)
#   train        cfg2 / cfg4 fused training-step times (bench.train_step_rate)
#   wide         cfg4 forward (k_wide) time
#   sweep        tools/batch_sweep.py loss / forward (2^16..2^24 rows)
#   mix          tools/ubench/mix_rate (VALU / MFMA co-issue rates)
#   calib        the calibrator-fit epoch variant (bench.calibrator_epoch_rate)
#   abbits       tools/ab/ab_bits.py (output fingerprints) for the shipped lib and every tools/ab/lib*.so
#   abtrace      tools/sgpr_trace.py for every tools/ab/lib*.so (trace builds) at AB_TRACE_B rows
#   abpower      tools/power_probe.py (board power, energy per row) for the shipped lib and every tools/ab/lib*.so
#   abil         tools/ab/ab_interleave.py: every tools/ab/lib*.so and the shipped lib, interleaved in one process
#   abwide       tools/ab/ab_wide_train.py (cfg4 training step) for the shipped lib and every tools/ab/lib*.so, x3
#   abvjp        tools/ab/ab_vjp.py (cfg2 training step + gradient checksum) for the shipped lib and every tools/ab/lib*.so, x3
#   abterms      tools/ab/ab_terms.py (loss-term bits + fp64 check) for every tools/ab/lib*.so
#   roctx        rocprofv3 marker + kernel trace of the roctx-ranged build (make roctx)
#   prof:<wl>:<mode>:<n>  kernel trace of tools/prof_target.py (clock settled first) and
#                tools/trace_stats.py over its last n calls
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  local t0=$(date +%s)
  timeout -k 10 "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc ($(( $(date +%s) - t0 ))s)"
  tail -n ${TAILN:-4} gpurun_out/$name.log | grep -v amdgpu.ids
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case "$step" in
    tests) TAILN=12 CNF_RECORD_DIR=gpurun_out run tests 600 python -u -m pytest tests -m gpu -q -rfs --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) TAILN=2 run bench 600 python bench.py ;;
    trace) CNF_TRACE_DUMP=gpurun_out/trace_loss.npz run trace_loss 180 python tools/sgpr_trace.py loss && CNF_TRACE_DUMP=gpurun_out/trace_fwd.npz run trace_fwd 180 python tools/sgpr_trace.py forward ;;
    rate) run rate 300 python tools/quick_rate.py loss forward inverse ;;
    train) run train 300 python -c "import json, torch, bench; d = torch.device('cuda:0'); print(json.dumps({w: bench.train_step_rate(d, w, steps=(20 if w == 'cfg2' else 5)) for w in ('cfg2', 'cfg4')}))" ;;
    wide) run wide 300 python -c "import json, torch, bench; d = torch.device('cuda:0'); r = bench.Runner(dict(bench.WORKLOADS['cfg4']), d, 1e9); t = min(bench.kernel_only_seconds(r, 10) for _ in range(3)); print(json.dumps({'cfg4_forward_us': round(t * 1e6, 1)}))" ;;
    sweep) run sweep_loss 300 python tools/batch_sweep.py loss && run sweep_fwd 300 python tools/batch_sweep.py forward ;;
    mix) run mix_rate 120 tools/ubench/mix_rate ;;
    calib) run calib 300 python -c "import json, torch, bench; print(json.dumps(bench.calibrator_epoch_rate(torch.device('cuda:0'))))" ;;
    ab)
      for lib in tools/ab/lib*.so; do
        [ -e "$lib" ] || continue
        n=$(basename "$lib" .so)
        TAILN=${AB_TAIL:-4} CNF_HIP_LIB=$PWD/$lib run "ab_$n" 300 python tools/quick_rate.py ${AB_MODE:-loss}
      done ;;
    abbits)
      run abbits_shipped 300 python tools/ab/ab_bits.py
      for lib in tools/ab/lib*.so; do
        [ -e "$lib" ] || continue
        n=$(basename "$lib" .so)
        CNF_HIP_LIB=$PWD/$lib run "abbits_$n" 300 python tools/ab/ab_bits.py
      done ;;
    abtrace)
      for lib in tools/ab/lib*.so; do
        [ -e "$lib" ] || continue
        n=$(basename "$lib" .so)
        for b in ${AB_TRACE_B:-1048576 8388608}; do
          TAILN=1 CNF_HIP_LIB=$PWD/$lib run "abtrace_${n}_$b" 180 python tools/sgpr_trace.py ${AB_MODE:-loss} $b
        done
      done ;;
    abpower)
      TAILN=1 run power_shipped 120 python tools/power_probe.py ${AB_MODE:-loss} 3 ${AB_B:-1048576}
      for lib in tools/ab/lib*.so; do
        [ -e "$lib" ] || continue
        n=$(basename "$lib" .so)
        TAILN=1 CNF_HIP_LIB=$PWD/$lib run "power_$n" 120 python tools/power_probe.py ${AB_MODE:-loss} 3 ${AB_B:-1048576}
      done ;;
    abil) TAILN=${AB_TAIL:-6} run abil 600 python tools/ab/ab_interleave.py ${AB_MODES:-loss,forward} ${AB_BS:-1048576,8388608} ${AB_ROUNDS:-9} ;;
    abwide)  # cfg4 training step per build, separate processes, shipped / builds interleaved
      for rep in 1 2 3; do
        TAILN=1 run abwide_shipped_$rep 300 python tools/ab/ab_wide_train.py
        for lib in tools/ab/lib*.so; do
          [ -e "$lib" ] || continue
          n=$(basename "$lib" .so)
          TAILN=1 CNF_HIP_LIB=$PWD/$lib run "abwide_${n}_$rep" 300 python tools/ab/ab_wide_train.py
        done
      done ;;
    abvjp)  # cfg2 training step per build, separate processes, shipped / builds interleaved
      for rep in 1 2 3; do
        TAILN=1 run abvjp_shipped_$rep 300 python tools/ab/ab_vjp.py
        for lib in tools/ab/lib*.so; do
          [ -e "$lib" ] || continue
          n=$(basename "$lib" .so)
          TAILN=1 CNF_HIP_LIB=$PWD/$lib run "abvjp_${n}_$rep" 300 python tools/ab/ab_vjp.py
        done
      done ;;
    abterms)
      for lib in tools/ab/lib*.so; do
        [ -e "$lib" ] || continue
        n=$(basename "$lib" .so)
        CNF_HIP_LIB=$PWD/$lib run "abterms_$n" 300 python tools/ab/ab_terms.py
      done ;;
    prof:*)  # prof:<workload>:<mode>:<launches> -> gpurun_out/prof_<workload>_<mode>/
      IFS=: read -r _ wl md nl <<< "$step"
      rm -rf gpurun_out/prof_${wl}_${md}
      run prof_${wl}_${md} 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${wl}_${md} -o run --output-format csv -- python tools/prof_target.py --workload $wl --mode $md --launches $nl &&
      python tools/trace_stats.py gpurun_out/prof_${wl}_${md}/run_kernel_trace.csv $nl gpurun_out/prof_${wl}_${md}/settled_stats.csv ;;
    roctx)  # the traced build's ranges beside its kernels (make roctx)
      rm -rf gpurun_out/roctx
      CNF_HIP_LIB=$PWD/calibration-normalizing-flows_amd/cnf_hip/libcnf_hip_roctx.so run roctx 300 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/roctx -o run --output-format csv -- python tools/prof_target.py --mode loss --launches 20 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
