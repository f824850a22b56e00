#!/bin/bash
# A/B of experimental library builds: tools/ab/ab_run.sh <script> <variant>...
# (each variant = cnf_hip/libcnf_hip_<variant>.so), one JSON line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
S=$1; shift
for v in "$@"; do
  CNF_HIP_LIB=$PWD/calibration-normalizing-flows_amd/cnf_hip/libcnf_hip_$v.so timeout -k 10 240 python $S >> gpurun_out/ab.log 2>&1
  rc=$?
  tail -n 1 gpurun_out/ab.log
  if [ $rc -ne 0 ]; then echo "stop: $v rc=$rc"; exit $rc; fi
done
