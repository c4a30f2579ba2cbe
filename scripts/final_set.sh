#!/bin/bash
# The round's measurement set on one box (TAG, default r06_v3): GPU suite + smoke, rocprofv3 kernel
# stats and read / write traffic per workload, SQ counter groups, then the bench lines.
#   TAG=r06_v3 bash scripts/final_set.sh   (outputs under gpurun_out/$TAG)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06_v3}
O=gpurun_out/$TAG
mkdir -p $O
TAG=$TAG STAGES="tests smoke" bash scripts/session.sh || exit $?
OUT=$O/ctr STAGE=traffic CFGS="${TCFGS:-cfg3 cfg3_bf16 cfg2 cfg5 cfg5_bf16 rfstate}" bash scripts/r4_counters.sh || exit $?
OUT=$O/ctr STAGE=sq CFGS="${SCFGS:-cfg3 cfg3_bf16 cfg5_bf16}" bash scripts/r4_counters.sh || exit $?
# summaries into profiles/ (copied under $O/profiles, the raw traces removed: gpurun copies back
# at most 64 MiB of gpurun_out/)
for c in ${TCFGS:-cfg3 cfg3_bf16 cfg2 cfg5 cfg5_bf16 rfstate}; do
  python3 scripts/r4_traffic.py $TAG $c $O/ctr > $O/traffic_$c.log 2>&1 || { echo "traffic summary $c failed"; tail -3 $O/traffic_$c.log; }
done
for c in ${SCFGS:-cfg3 cfg3_bf16 cfg5_bf16}; do
  ks=profiles/${TAG}_kernel_stats_$c.csv; [ $c = cfg3 ] && ks=profiles/${TAG}_kernel_stats.csv
  python3 scripts/r4_ctr_summary.py $c $O/ctr $ks $TAG > $O/ctr_$c.log 2>&1 || { echo "counter summary $c failed"; tail -3 $O/ctr_$c.log; }
done
mkdir -p $O/profiles && cp profiles/${TAG}_* $O/profiles/ 2>/dev/null
rm -rf $O/ctr
for c in ${BCFGS:-cfg3 cfg5 cfg2 rfstate}; do
  echo "== bench $c"
  timeout -k 10 400 python3 bench.py --config $c > $O/bench_$c.log 2>&1; rc=$?
  echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' $O/bench_$c.log > $O/bench_$c.json
done
echo FINAL_SET_DONE
