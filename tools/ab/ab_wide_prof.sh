#!/bin/bash
# rocprof kernel stats of the cfg4 training step for every tools/ab/libw*.so
# (make ab ABSRC=cnf_wide16 ...): per lib, the step time and the average
# duration of the fused sweeps' kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for lib in tools/ab/${AB_GLOB:-libw*}.so; do
  n=$(basename "$lib" .so)
  rm -rf gpurun_out/abp_$n
  CNF_HIP_LIB=$PWD/$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$n -o run \
    --output-format csv -- python tools/ab/ab_wide_train.py > gpurun_out/abp_$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(grep '"ms"' gpurun_out/abp_$n.log)"
  python3 - "$n" << 'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/abp_%s/**/run_kernel_stats.csv" % sys.argv[1], recursive=True)
for r in csv.DictReader(open(f[0])) if f else []:
    if any(k in r["Name"] for k in ("k_wtrain16", "k_wdw16", "k_reduce_cols")):
        print("   %-40s %8.1f us x %s" % (r["Name"].split("(anonymous namespace)::")[-1][:40], float(r["AverageNs"]) / 1e3, r["Calls"]))
PY
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
