#!/bin/bash
# round-4 GPU session 27: GPU suite; the LDS-DMA token GEMM on the fp32 path (3-part split on the
# fragment read) against the register-staged fp32 kernel (MEP_TGEMM_DMA=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t27.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t27.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t27.log | head -20
[ $rc -eq 0 ] || exit $rc
V="dma=X=1;reg=MEP_TGEMM_DMA=0"
TAG=s27c5 REPS=2 STEPS=30 ARGS="--config cfg5 --dtype fp32" VARIANTS="$V" bash scripts/r4_ab.sh > gpurun_out/s27.log 2>&1 || { tail -5 gpurun_out/s27.log; exit 1; }
python3 - <<'PY'
import json
for t in ('s27c5',):
    for l in open('gpurun_out/r4ab_%s.jsonl' % t):
        d=json.loads(l); k=d['kernels']
        print(t, d['ab'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'tgemm' in n})
PY
echo ALLDONE
