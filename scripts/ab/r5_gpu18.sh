#!/bin/bash
# round-5 GPU session 18 (rerun 2: guard-free products, fragment ring, batched fill): the LDS-resident token GEMM (mep_wgemm_ws) -- kernel tests (bit-equal to
# mep_wgemm), the realformer suite, then rfstate / cfg2 with MEP_WGEMM_WS=1 / 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rfw.py tests/test_gpu_realformer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t18.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t18.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t18.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    for c in rfstate cfg2; do
    MEP_WGEMM_WS=$v timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b18_${v}_$c.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5_b18_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b18_%s_%s.log'%(sys.argv[1],sys.argv[2])).read().strip().splitlines()[-1])
k=d['kernels']
g=k.get('mep_wgemm_ws') or k.get('mep_wgemm')
print('ws=%s'%sys.argv[1], sys.argv[2], d['ms_per_step'], 'gemm/step %.1f us (%d launches)' % (g['ms_per_step']*1e3, g['launches_per_step']))
PY
    done
  done
done
echo ALLDONE
