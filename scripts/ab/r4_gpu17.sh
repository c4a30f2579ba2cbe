#!/bin/bash
# round-4 GPU session 17: GPU suite; LayerNorm kernels templated on features per lane
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t17.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t17.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t17.log | head -20
[ $rc -eq 0 ] || exit $rc
TAG=s17c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="base=X=1" bash scripts/r4_ab.sh || exit $?
python3 - <<'PY'
import json
for l in open('gpurun_out/r4ab_s17c5bf.jsonl'):
    d=json.loads(l); k=d['kernels']
    print({n: round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if n in ('mep_layernorm_fwd','mep_layernorm_bwd','mep_sum_rows','mep_pool_fwd','mep_head_fwd_bwd','mep_reduce_grads','mep_clip_adam_ext')})
PY
echo ALLDONE
