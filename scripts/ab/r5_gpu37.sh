#!/bin/bash
# round-5 GPU session 37: bf16 epilogues at 12 waves per workgroup (one tile per wave at one
# workgroup per CU) -- parity of the variant (bf16 + pool-fold tests), then
# cfg3 bench lines (fp32 headline + nested bf16) default / eb12 / efb12, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MEP_LIB=$PWD/variants/efb12/libmep_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_pool_fold.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t37.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t37.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t37.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in def eb12 efb12; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/r5_b37_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b37_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b37_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
b=d['bf16']; k=b['kernels']
g=lambda n: k[n]['avg_launch_us'] if n in k else 0
print('%-6s fp32 %.4f  bf16 %.4f ms  epi_fwd %.1f  epi_bwd %.1f' % (sys.argv[1], d['ms_per_step'], b['ms_per_step'], g('mep_block_epi_fwd'), g('mep_block_epi_bwd')))
PY
  done
done
echo ALLDONE
