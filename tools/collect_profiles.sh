#!/bin/bash
# Copy one gpu_check.sh session's summaries from gpurun_out/ into profiles/
# (tracked): kernel-trace stats per pass, PMC medians, HBM traffic per launch,
# and the bench line.  usage: tools/collect_profiles.sh TAG
set -eu
TAG=$1
cd "$(dirname "$0")/.."
mkdir -p profiles
cp gpurun_out/prof_${TAG}/run_kernel_stats.csv profiles/${TAG}_bench_kernel_stats.csv
[ -f gpurun_out/prof_${TAG}/settled_stats.csv ] && cp gpurun_out/prof_${TAG}/settled_stats.csv profiles/${TAG}_bench_settled_stats.csv
for d in gpurun_out/prof_${TAG}_*; do
  n=${d#gpurun_out/prof_${TAG}_}
  [ -f $d/run_kernel_stats.csv ] && cp $d/run_kernel_stats.csv profiles/${TAG}_${n}_kernel_stats.csv
  [ -f $d/settled_stats.csv ] && cp $d/settled_stats.csv profiles/${TAG}_${n}_settled_stats.csv
done
for m in loss fwd; do
  [ -f gpurun_out/sweep_$m.log ] && grep '^{' gpurun_out/sweep_$m.log > profiles/${TAG}_batch_sweep_$m.jsonl
done
for spec in "cfg2 loss k_sgpr 1048576" "cfg2 all k_valu 1048576" "cfg2 train k_vjp2 1048576" "cfg4 forward k_wide16 262144" "cfg4 train k_wdw16 262144" "cfg4 train k_wtrain16_fwd 262144" "cfg4 train k_wtrain16_bwd 262144"; do
  set -- $spec
  dir=gpurun_out/pmc_${TAG}_$1_$2_$1
  [ -d $dir ] || continue
  sfx=$1_$2; case "$3" in k_wtrain16*) sfx=$1_$2_$3;; esac
  python tools/pmc_summary.py $dir $3 > profiles/${TAG}_pmc_${sfx}.txt
  python tools/pmc_traffic.py $dir profiles/${TAG}_traffic_${sfx}.json $1 $4 $3 > /dev/null
done
for rec in inverse_errors predict_errors; do
  [ -f gpurun_out/$rec.jsonl ] && cp gpurun_out/$rec.jsonl profiles/${TAG}_$rec.jsonl
done
grep '^{"metric"' gpurun_out/bench.log | tail -1 >> profiles/${TAG}_bench.jsonl
ls profiles/ | grep "^${TAG}_"
