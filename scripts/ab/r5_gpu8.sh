#!/bin/bash
# round-5 GPU session 8: single-phase fp32 epilogue forward (epi_fwd_wp2r): GPU suite, then the cfg3
# fp32 step A/B against the two-phase kernel (variants/twophase)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t8.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t8.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t8.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in main twophase; do
    if [ $v = main ]; then L=""; else L=variants/$v/libmep_hip.so; fi
    MEP_LIB=$L timeout -k 10 200 python3 bench.py --no-bf16 --no-cpu-baseline --no-probe > gpurun_out/r5_b8_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5_b8_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b8_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'epi_fwd', d['kernels']['mep_block_epi_fwd']['avg_launch_us'], 'sum', d['kernels_sum_ms'])
PY
  done
done
echo ALLDONE
