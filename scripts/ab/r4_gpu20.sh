#!/bin/bash
# round-4 GPU session 20: GPU suite (with the LDS-DMA bf16 token GEMM); cfg5 bf16 A/B of
# MEP_TGEMM_DMA=1 (default) against the register-staged bf16 kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t20.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t20.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t20.log | head -20
[ $rc -eq 0 ] || exit $rc
TAG=s20c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="dma=X=1;reg=MEP_TGEMM_DMA=0" bash scripts/r4_ab.sh || exit $?
python3 - <<'PY'
import json
for l in open('gpurun_out/r4ab_s20c5bf.jsonl'):
    d=json.loads(l); k=d['kernels']
    print(d['ab'], d['ms_per_step'], {n: round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'tgemm' in n})
PY
echo ALLDONE
