#!/bin/bash
# round-4 GPU session 24: GPU suite; weight-gradient chunk chosen over 1-4 rounds of resident
# workgroups (base) against one round (MEP_WG_SETUP_TOKENS=1000000)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t24.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t24.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t24.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;one=MEP_WG_SETUP_TOKENS=1000000"
TAG=s24c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh > gpurun_out/s24.log 2>&1 || { tail -5 gpurun_out/s24.log; exit 1; }
TAG=s24c5 REPS=2 STEPS=30 ARGS="--config cfg5 --dtype fp32" VARIANTS="$V" bash scripts/r4_ab.sh >> gpurun_out/s24.log 2>&1 || { tail -5 gpurun_out/s24.log; exit 1; }
TAG=s24c3 REPS=2 STEPS=100 ARGS="--config cfg3 --dtype fp32" VARIANTS="$V" bash scripts/r4_ab.sh >> gpurun_out/s24.log 2>&1 || { tail -5 gpurun_out/s24.log; exit 1; }
python3 - <<'PY'
import json
for t in ('s24c5bf','s24c5','s24c3'):
    for l in open('gpurun_out/r4ab_%s.jsonl' % t):
        d=json.loads(l); k=d['kernels']
        print(t, d['ab'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'wgrad' in n or 'reduce' in n})
PY
echo ALLDONE
