#!/bin/bash
# One rank through the RCCL NLL all-reduce path of bench.py (--dist-check: the
# overlapped and synchronous forms timed side by side) for several bucket sizes.
# Lines: gpurun_out/dist_check.jsonl.  usage: tools/dist_check.sh [buckets...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/dist_check.jsonl
for b in ${@:-50 1}; do
  timeout -k 10 200 python bench.py --dist-check --no-variants --no-cpu-baseline --nll-bucket $b \
    > gpurun_out/dist_check_$b.log 2>&1 || { tail -5 gpurun_out/dist_check_$b.log; exit 1; }
  python - "$b" << 'PY'
import json, sys
line = [l for l in open("gpurun_out/dist_check_%s.log" % sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
r = {"nll_bucket": int(sys.argv[1]), "ms_per_step": d["ms_per_step"], "dist_check": d["dist_check"],
     "kernel_us": d["rank_kernel_us"]}
print(json.dumps(r))
open("gpurun_out/dist_check.jsonl", "a").write(json.dumps(r) + "\n")
PY
done
