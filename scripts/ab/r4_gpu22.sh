#!/bin/bash
# round-4 GPU session 22: cfg3 bf16 unify on the LDS-DMA token GEMM (MEP_TGEMM_MIN_K=0; 128 or 64
# tokens per workgroup) against mep_unify
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V="base=X=1;tg=MEP_TGEMM_MIN_K=0;tg64=MEP_TGEMM_MIN_K=0 MEP_LIB=$PWD/variants/tt1/libmep_hip.so"
TAG=s22c3bf REPS=3 STEPS=100 ARGS="--config cfg3 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh > gpurun_out/s22.log 2>&1 || { tail -5 gpurun_out/s22.log; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r4ab_s22c3bf.jsonl'):
    d=json.loads(l); k=d['kernels']
    print(d['ab'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'tgemm' in n or 'unify' in n})
PY
echo ALLDONE
