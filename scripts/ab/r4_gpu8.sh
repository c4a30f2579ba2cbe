#!/bin/bash
# round-4 GPU session 8: GPU suite; A/B of the bf16 weight-gradient prefetch depth (variants/sl3, sl4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t8.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t8.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t8.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;sl3=MEP_LIB=variants/sl3/libmep_hip.so;sl4=MEP_LIB=variants/sl4/libmep_hip.so"
TAG=s8c3bf REPS=2 ARGS="--dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
TAG=s8c5bf REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
