# SQ + L2 counter groups (one rocprofv3 pass each, kernel trace only) for the realformer State_Transfer
# workload (and cfg3 unless CFGS says otherwise), summarised on the box into profiles/<TAG>_counters_<cfg>.*
#   TAG=r06_l2 CFGS="rfstate cfg3" bash scripts/l2_counters.sh
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
TAG=${TAG:-r06_l2}
CFGS=${CFGS:-rfstate cfg3}
O=gpurun_out/$TAG; mkdir -p $O
for c in $CFGS; do
  case $c in cfg3) A="--config cfg3 --dtype fp32";; *) A="--config $c";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${c}_trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bf16 --no-probe $A > $O/trace_$c.log 2>&1 || exit 1
  cp $(find $O/${c}_trace -name "*kernel_stats.csv" | head -1) $O/ks_$c.csv
done
OUT=$O/ctr STAGE=sq SQ_L2=1 CFGS="$CFGS" bash scripts/r4_counters.sh || exit 1
for c in $CFGS; do
  python3 scripts/r4_ctr_summary.py $c $O/ctr $O/ks_$c.csv $TAG > $O/sum_$c.log 2>&1
  cp profiles/${TAG}_counters_$c.* $O/
done
rm -rf $O/ctr $O/*_trace
