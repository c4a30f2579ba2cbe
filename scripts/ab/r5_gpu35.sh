#!/bin/bash
# round-5 GPU session 35: mep_wgemm_sum (cfg2's input-gradient GEMMs + per-modality sum in one
# launch) -- its parity tests, then the cfg2 bench with the fused path on / off, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rfw.py tests/test_gpu_realformer.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t35.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t35.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t35.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    MEP_RF_WGEMM_SUM=$v timeout -k 10 300 python3 bench.py --config cfg2 --no-cpu-baseline --no-probe > gpurun_out/r5_b35_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b35_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b35_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('kernels', {})
print('wgemm_sum=%s %.4f ms  %s' % (sys.argv[1], d['ms_per_step'], {n: v.get('avg_launch_us') for n, v in k.items() if 'sum' in n or 'wgemm' in n}))
PY
  done
done
echo ALLDONE
