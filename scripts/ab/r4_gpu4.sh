#!/bin/bash
# round-4 GPU session 4: GPU suite, then same-box A/B of the forward-attention / unify-staging
# changes against the previous attention object (variants/prev)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t4.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t4.log | head -20
[ $rc -eq 0 ] || exit $rc
TAG=fwd3bf REPS=2 ARGS="--dtype bf16" VARIANTS="base=X=1;prev=MEP_LIB=variants/prev/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
TAG=fwd3 REPS=1 ARGS="--dtype fp32" VARIANTS="base=X=1;prev=MEP_LIB=variants/prev/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
TAG=fwd5bf REPS=1 ARGS="--config cfg5 --dtype bf16" STEPS=30 VARIANTS="base=X=1;prev=MEP_LIB=variants/prev/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
