#!/bin/bash
# round-5 GPU session 28: epilogue weight images (mep_epi_images once per step, LDS-DMA copy-in)
# -- full GPU suite, then cfg3 (fp32 + bf16) and cfg5 with MEP_EPI_IMAGE=1 / 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t28.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t28.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t28.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    for c in cfg3 cfg5; do
      MEP_EPI_IMAGE=$v timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b28_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b28_${v}_$c.log; exit 1; }
      python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b28_%s_%s.log'%(sys.argv[1],sys.argv[2])).read().strip().splitlines()[-1])
b=d.get('bf16') or {}
g=lambda x, n: x[n]['avg_launch_us'] if n in x else 0
f=lambda x: 'fwd %.1f bwd %.1f img %.1f' % (g(x,'mep_block_epi_fwd'), g(x,'mep_block_epi_bwd'), g(x,'mep_epi_images'))
print('img=%s'%sys.argv[1], sys.argv[2], 'fp32', d['ms_per_step'], f(d['kernels']), '| bf16', b.get('ms_per_step'), f(b['kernels']) if b else '')
PY
    done
  done
done
echo ALLDONE
