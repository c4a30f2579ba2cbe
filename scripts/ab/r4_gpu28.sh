#!/bin/bash
# round-4 GPU session 28: GPU suite; 16-byte column-quad pooling forward (base) against the 4-byte
# form (variants/pold, MEP_POOL_V4=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t28.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t28.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t28.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;pold=MEP_LIB=$PWD/variants/pold/libmep_hip.so"
TAG=s28c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh > gpurun_out/s28.log 2>&1 || { tail -5 gpurun_out/s28.log; exit 1; }
TAG=s28c3bf REPS=2 STEPS=100 ARGS="--config cfg3 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh >> gpurun_out/s28.log 2>&1 || { tail -5 gpurun_out/s28.log; exit 1; }
python3 - <<'PY'
import json
for t in ('s28c5bf','s28c3bf'):
    for l in open('gpurun_out/r4ab_%s.jsonl' % t):
        d=json.loads(l); k=d['kernels']
        print(t, d['ab'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'pool' in n})
PY
echo ALLDONE
