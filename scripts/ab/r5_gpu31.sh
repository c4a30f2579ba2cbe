#!/bin/bash
# round-5 GPU session 31: epilogue products with A fragments read MEP_TG_RING steps ahead (2 =
# main, 3, 4, 0 = the grouped reads) -- cmu / bf16 / ren parity, then cfg3 and cfg5 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cmu.py tests/test_gpu_bf16.py tests/test_gpu_ren.py tests/test_gpu_pool_fold.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t31.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t31.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t31.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in main ring3 ring4 ring0; do
    if [ $v = main ]; then L=""; else L=variants/$v/libmep_hip.so; fi
    for c in cfg3 cfg5; do
      MEP_LIB=$L timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b31_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b31_${v}_$c.log; exit 1; }
      python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b31_%s_%s.log'%(sys.argv[1],sys.argv[2])).read().strip().splitlines()[-1])
b=d.get('bf16') or {}
g=lambda x, n: x[n]['avg_launch_us'] if n in x else 0
f=lambda x: 'fwd %.1f bwd %.1f' % (g(x,'mep_block_epi_fwd'), g(x,'mep_block_epi_bwd'))
print('%-6s'%sys.argv[1], sys.argv[2], 'fp32', d['ms_per_step'], f(d['kernels']), '| bf16', b.get('ms_per_step'), f(b['kernels']) if b else '')
PY
    done
  done
done
echo ALLDONE
