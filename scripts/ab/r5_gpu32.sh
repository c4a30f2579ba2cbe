#!/bin/bash
# round-5 GPU session 32: LayerNorm parameters staged in LDS by the single-phase epilogues, the fp32
# forward's next q rows issued before the stores (no
# global load at every tile's end) -- parity, then cfg3 / cfg5 lines (compare session 31 main)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cmu.py tests/test_gpu_bf16.py tests/test_gpu_ren.py tests/test_gpu_pool_fold.py tests/test_gpu_cfg5_shape.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t32.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t32.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t32.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for c in cfg3 cfg5; do
    timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b32_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b32_$c.log; exit 1; }
    python3 - $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b32_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
b=d.get('bf16') or {}
g=lambda x, n: x[n]['avg_launch_us'] if n in x else 0
f=lambda x: 'fwd %.1f bwd %.1f' % (g(x,'mep_block_epi_fwd'), g(x,'mep_block_epi_bwd'))
print(sys.argv[1], 'fp32', d['ms_per_step'], f(d['kernels']), '| bf16', b.get('ms_per_step'), f(b['kernels']) if b else '')
PY
  done
done
echo ALLDONE
