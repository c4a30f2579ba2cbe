#!/bin/bash
# round-4 GPU session 21: GPU suite; LDS-only barriers in the wide attention backward and the DMA
# token GEMM (base) against __syncthreads (nolb), staging ring depth 3 / 4, 4 X chunks in the GEMM
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t21.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t21.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t21.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1"
for n in nolb ns3 ns4 tgpfx4; do V="$V;$n=MEP_LIB=$PWD/variants/$n/libmep_hip.so"; done
TAG=s21c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh > gpurun_out/s21.log 2>&1 || { tail -5 gpurun_out/s21.log; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r4ab_s21c5bf.jsonl'):
    d=json.loads(l); k=d['kernels']
    print(d['ab'], d['ms_per_step'], {n.replace('mep_',''): round(1e3*v['ms_per_step']/max(1,v['launches_per_step']),1) for n,v in k.items() if 'tgemm' in n or 'attn' in n})
PY
echo ALLDONE
