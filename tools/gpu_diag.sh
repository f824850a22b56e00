#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS=1,4 timeout -k 10 300 python tools/bench_variants.py > gpurun_out/diag_real.log 2>&1; echo "real rc=$?"; cat gpurun_out/diag_real.log
VARIANTS=1,4 CNF_HIP_LIB=$PWD/calibration-normalizing-flows_amd/cnf_hip/libcnf_hip_diag.so timeout -k 10 300 python tools/bench_variants.py > gpurun_out/diag_fake.log 2>&1; echo "fake rc=$?"; cat gpurun_out/diag_fake.log
