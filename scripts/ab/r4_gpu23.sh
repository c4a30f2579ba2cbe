#!/bin/bash
# round-4 GPU session 23: weight-gradient workgroup count (MEP_WG_TARGET) on the bf16 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V="base=X=1;t384=MEP_WG_TARGET=384;t512=MEP_WG_TARGET=512;t768=MEP_WG_TARGET=768"
TAG=s23c3bf REPS=2 STEPS=100 ARGS="--config cfg3 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh > gpurun_out/s23.log 2>&1 || { tail -5 gpurun_out/s23.log; exit 1; }
TAG=s23c5bf REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh >> gpurun_out/s23.log 2>&1 || { tail -5 gpurun_out/s23.log; exit 1; }
python3 - <<'PY'
import json
for t in ('s23c3bf','s23c5bf'):
    for l in open('gpurun_out/r4ab_%s.jsonl' % t):
        d=json.loads(l); k=d['kernels']
        print(t, d['ab'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'wgrad' in n or 'reduce' in n})
PY
echo ALLDONE
