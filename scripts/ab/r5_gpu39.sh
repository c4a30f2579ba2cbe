#!/bin/bash
# round-5 GPU session 39: epilogue prologues with every load issued before the first LDS write
# (MEP_EPI_PROLOGUE) -- parity (epilogue / bf16 / cmu tests), the phase trace, then cfg3 and cfg5
# bench lines against the per-weight staging (variant noprol), twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_pool_fold.py tests/test_gpu_cmu.py tests/test_gpu_encoders.py tests/test_gpu_ren.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t39.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t39.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t39.log | head -20
[ $rc -eq 0 ] || exit $rc
MEP_LIB=$PWD/variants/etrace/libmep_hip.so timeout -k 10 300 python3 scripts/epi_trace1.py > gpurun_out/r5_trace39.log 2>&1 || { echo trace failed; tail -5 gpurun_out/r5_trace39.log; exit 1; }
tail -4 gpurun_out/r5_trace39.log
for rep in 1 2; do
  for v in def noprol; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    for c in cfg3 cfg5; do
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b39_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b39_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b39_%s_%s.log'%(sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
b=d['bf16']
g=lambda x, n: x['kernels'][n]['avg_launch_us'] if n in x['kernels'] else 0
print('%-6s %s fp32 %.4f (fwd %.1f bwd %.1f)  bf16 %.4f (fwd %.1f bwd %.1f)' % (sys.argv[1], sys.argv[2], d['ms_per_step'], g(d,'mep_block_epi_fwd'), g(d,'mep_block_epi_bwd'), b['ms_per_step'], g(b,'mep_block_epi_fwd'), g(b,'mep_block_epi_bwd')))
PY
    done
  done
done
echo ALLDONE
