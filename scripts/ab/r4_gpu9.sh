#!/bin/bash
# round-4 GPU session 9: GPU suite; A/B of the bf16 backward delta on the matrix core against HEAD (variants/hd)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t9.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t9.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t9.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;hd=MEP_LIB=variants/hd/libmep_hip.so"
TAG=s9c3bf REPS=2 ARGS="--dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
TAG=s9c5bf REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
