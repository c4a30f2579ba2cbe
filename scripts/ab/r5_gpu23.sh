#!/bin/bash
# round-5 GPU session 23: attention dq rows cleared by the forward epilogues (no fill kernel)
# -- kernel + realformer tests, the rfstate / cfg2 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rfw.py tests/test_gpu_realformer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t23.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t23.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t23.log | head -20
[ $rc -eq 0 ] || exit $rc
for c in rfstate cfg2; do
  timeout -k 10 300 python3 bench.py --config $c --no-probe > gpurun_out/r5_b23_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/r5_b23_$c.log; exit 1; }
  python3 - $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b23_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], {k: v['avg_launch_us'] for k, v in d['kernels'].items() if 'gemm' in k}, d['roofline']['kernel'], d['roofline']['frac'])
PY
done
echo ALLDONE
