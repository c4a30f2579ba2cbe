#!/bin/bash
# round-4 GPU session 26: GPU suite; per-modality sums on 32-bit indices, no per-step row0 fill
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t26.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t26.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t26.log | head -20
[ $rc -eq 0 ] || exit $rc
TAG=s26c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="base=X=1" bash scripts/r4_ab.sh > gpurun_out/s26.log 2>&1 || { tail -5 gpurun_out/s26.log; exit 1; }
TAG=s26c3bf REPS=2 STEPS=100 ARGS="--config cfg3 --dtype bf16" VARIANTS="base=X=1" bash scripts/r4_ab.sh >> gpurun_out/s26.log 2>&1 || { tail -5 gpurun_out/s26.log; exit 1; }
python3 - <<'PY'
import json
for t in ('s26c5bf','s26c3bf'):
    for l in open('gpurun_out/r4ab_%s.jsonl' % t):
        d=json.loads(l); k=d['kernels']
        print(t, d['ab'], d['value'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'sum' in n})
PY
echo ALLDONE
