#!/bin/bash
# PMC counter passes (each its own rocprofv3 run, --kernel-trace only beside --pmc).
# usage: gpu_pmc.sh TAG WORKLOAD "extra prof_target args" "pass1 counters" "pass2 counters" ...
set -u
TAG=$1; WL=$2; EXTRA=$3; shift 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_${TAG}_${WL}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $OUT/p$i -o run --output-format csv -- python tools/prof_target.py --workload $WL $EXTRA > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $ctrs"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; fi
  # a rejected counter list (rc 1/2) is reported and skipped; anything else ends the run
  if [ $rc -gt 2 ]; then exit $rc; fi
done
exit 0
