#!/bin/bash
# round-4 GPU session 10: tgemm / unify tests; A/B of the tgemm chunk pipeline depth (variants/pfN)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tgemm.py tests/test_gpu_ren.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t10.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t10.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t10.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;pf2=MEP_LIB=variants/pf2/libmep_hip.so;pf3=MEP_LIB=variants/pf3/libmep_hip.so;pf6=MEP_LIB=variants/pf6/libmep_hip.so"
TAG=s10c5bf REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
TAG=s10c5 REPS=1 STEPS=20 ARGS="--config cfg5 --dtype fp32" VARIANTS="base=X=1;pf2=MEP_LIB=variants/pf2/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
