#!/bin/bash
# Experiment session: GPU tests (default + persistent variants), then variant A/B.
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
  tail -n ${TAILN:-6} gpurun_out/$name.log | grep -v amdgpu.ids
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run pytest_gpu 900 python -m pytest tests -m gpu -q


VARIANTS=${VARIANTS:-0,1,2,3,4,5,6} TAILN=40 run variants 600 python tools/bench_variants.py
TAILN=30 VARIANTS=2,3 run scaling 400 python tools/bench_scaling.py
exit 0
