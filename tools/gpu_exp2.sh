#!/bin/bash
# variant A/B after the loss rewrite + VALU/LDS/SALU activity counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CASES=cfg2_loss,cfg2 VARIANTS=98 timeout -k 10 400 python tools/bench_variants.py > gpurun_out/variants2.log 2>&1
rc=$?; cat gpurun_out/variants2.log; [ $rc -ne 0 ] && exit $rc
exit 0
