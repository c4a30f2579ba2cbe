#!/bin/bash
# round-4 GPU session 5: GPU suite, A/B of the forward row-sum / permlane reductions and the bf16
# unify restructure
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t5.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t5.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t5.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;nomf=MEP_LIB=variants/nomf/libmep_hip.so;gprev=MEP_LIB=variants/gprev/libmep_hip.so;pp4=MEP_LIB=variants/pp4/libmep_hip.so;pp6=MEP_LIB=variants/pp6/libmep_hip.so"
TAG=s5c3bf REPS=2 ARGS="--dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
TAG=s5c5bf REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="base=X=1;nomf=MEP_LIB=variants/nomf/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
