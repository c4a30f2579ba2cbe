#!/bin/bash
# round-5 GPU session 24: block-weight gradients on a side stream concurrent with the attention
# backward (MEP_OVERLAP_WGRAD) -- full GPU suite, then cfg3 / cfg5 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t24.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t24.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t24.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    for c in cfg3 cfg5; do
      MEP_OVERLAP_WGRAD=$v timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b24_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b24_${v}_$c.log; exit 1; }
      python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b24_%s_%s.log'%(sys.argv[1],sys.argv[2])).read().strip().splitlines()[-1])
b=d.get('bf16') or {}
print('ovl=%s'%sys.argv[1], sys.argv[2], 'fp32', d['ms_per_step'], 'bf16', b.get('ms_per_step'), 'wgrad', d['kernels']['mep_wgrad'], 'attn_bwd', d['kernels']['mep_attn_bwd']['avg_launch_us'])
PY
    done
  done
done
echo ALLDONE
