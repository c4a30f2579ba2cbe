#!/bin/bash
# round-4 GPU session 30: GPU suite; fp32 attention forward with the mask term as the score
# accumulator's initial value (variants/mif) against the scale / subtract form (base)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MEP_LIB=$PWD/variants/mif/libmep_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t30.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t30.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t30.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;mif=MEP_LIB=$PWD/variants/mif/libmep_hip.so"
TAG=s30c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype fp32" VARIANTS="$V" bash scripts/r4_ab.sh > gpurun_out/s30.log 2>&1 || { tail -5 gpurun_out/s30.log; exit 1; }
TAG=s30c3bf REPS=2 STEPS=100 ARGS="--config cfg3 --dtype fp32" VARIANTS="$V" bash scripts/r4_ab.sh >> gpurun_out/s30.log 2>&1 || { tail -5 gpurun_out/s30.log; exit 1; }
python3 - <<'PY'
import json
for t in ('s30c5bf','s30c3bf'):
    for l in open('gpurun_out/r4ab_%s.jsonl' % t):
        d=json.loads(l); k=d['kernels']
        print(t, d['ab'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'attn' in n})
PY
echo ALLDONE
