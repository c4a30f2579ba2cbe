#!/bin/bash
# round-5 GPU session 40: the pool upstream's mean division out of line (it was evaluated for every
# element and selected away on the pool_T < 0 path) -- parity, then cfg3 against HEAD's build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_pool_fold.py tests/test_gpu_cmu.py tests/test_gpu_encoders.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t40.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t40.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t40.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in def base; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/r5_b40_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b40_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b40_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
b=d['bf16']
g=lambda x, n: x['kernels'][n]['avg_launch_us'] if n in x['kernels'] else 0
print('%-5s fp32 %.4f (fwd %.1f bwd %.1f)  bf16 %.4f (fwd %.1f bwd %.1f)' % (sys.argv[1], d['ms_per_step'], g(d,'mep_block_epi_fwd'), g(d,'mep_block_epi_bwd'), b['ms_per_step'], g(b,'mep_block_epi_fwd'), g(b,'mep_block_epi_bwd')))
PY
  done
done
echo ALLDONE
