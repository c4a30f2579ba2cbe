#!/bin/bash
# round-4 GPU session 29: GPU suite; bf16 attention forward with the mask term as the score
# accumulator's initial value (base) against the scale / subtract form (variants/nomi)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t29.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t29.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t29.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;nomi=MEP_LIB=$PWD/variants/nomi/libmep_hip.so"
TAG=s29c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh > gpurun_out/s29.log 2>&1 || { tail -5 gpurun_out/s29.log; exit 1; }
TAG=s29c3bf REPS=2 STEPS=100 ARGS="--config cfg3 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh >> gpurun_out/s29.log 2>&1 || { tail -5 gpurun_out/s29.log; exit 1; }
python3 - <<'PY'
import json
for t in ('s29c5bf','s29c3bf'):
    for l in open('gpurun_out/r4ab_%s.jsonl' % t):
        d=json.loads(l); k=d['kernels']
        print(t, d['ab'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'attn' in n})
PY
echo ALLDONE
