#!/bin/bash
# round-5 GPU session 42: end-of-round profiles (mep_wgemm_sum, 12-wave bf16 epilogues, out-of-line pool division, 24-bit row addressing) -- per workload the rocprofv3 kernel
# trace + stats, the 32-B read-unit and WRITE_SIZE passes (scripts/r4_counters.sh STAGE=traffic),
# the SQ groups of cfg3 (fp32, bf16); summarised on the box into profiles/r05_v3_* (raw CSVs
# dropped), then the bench lines of every workload, whose traffic fields cite those passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_t42.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t42.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/r5_t42.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke42.log 2>&1; rc=$?; tail -2 gpurun_out/r5_smoke42.log; [ $rc -eq 0 ] || exit $rc
R=gpurun_out/r5ctr
OUT=$R STAGE=traffic CFGS="cfg3 cfg3_bf16 cfg5 cfg5_bf16 cfg2 rfstate" PSTEPS=20 bash scripts/r4_counters.sh || exit $?
OUT=$R STAGE=sq CFGS="cfg3 cfg3_bf16" bash scripts/r4_counters.sh || exit $?
for c in cfg3 cfg3_bf16 cfg5 cfg5_bf16 cfg2 rfstate; do python3 scripts/r4_traffic.py r05_v3 $c $R > $R/sum_$c.txt || exit 1; done
python3 scripts/r4_ctr_summary.py cfg3 $R profiles/r05_v3_kernel_stats.csv r05 || exit 1
python3 scripts/r4_ctr_summary.py cfg3_bf16 $R profiles/r05_v3_kernel_stats_cfg3_bf16.csv r05 || exit 1
mkdir -p gpurun_out/p7
cp profiles/r05_* gpurun_out/p7/
rm -rf $R
timeout -k 10 300 python3 bench.py > gpurun_out/p7/r05_v3_bench_cfg3.json 2> gpurun_out/p7/err_cfg3.log || exit 1
for c in cfg5 cfg2 rfstate; do
  timeout -k 10 300 python3 bench.py --config $c > gpurun_out/p7/r05_v3_bench_$c.json 2> gpurun_out/p7/err_$c.log || exit 1
done
ls gpurun_out/p7
echo ALLDONE
