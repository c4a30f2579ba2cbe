cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r06_s21; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rfstate_trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bf16 --no-probe --config rfstate > $O/trace.log 2>&1 || exit 1
cp $(find $O/rfstate_trace -name "*kernel_stats.csv" | head -1) $O/ks_rfstate.csv
OUT=$O/ctr STAGE=sq SQ_L2=1 CFGS="rfstate cfg3" bash scripts/r4_counters.sh || exit 1
python3 scripts/r4_ctr_summary.py rfstate $O/ctr $O/ks_rfstate.csv r06_l2 > $O/sum_rfstate.log 2>&1
python3 scripts/r4_ctr_summary.py cfg3 $O/ctr profiles/r06_v3_kernel_stats.csv r06_l2 > $O/sum_cfg3.log 2>&1
cp profiles/r06_l2_counters_* $O/
rm -rf $O/ctr $O/rfstate_trace
