#!/bin/bash
# round-4 GPU session 11: GPU suite (ABI 3: dropout keep bits); A/B against the backward re-hashing
# the masks (variants/nobits)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t11.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t11.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t11.log | head -20
[ $rc -eq 0 ] || exit $rc
V="base=X=1;nobits=MEP_LIB=variants/nobits/libmep_hip.so"
TAG=s11c5bf REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
TAG=s11c5 REPS=1 STEPS=20 ARGS="--config cfg5 --dtype fp32" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
TAG=s11c3 REPS=2 ARGS="--dtype fp32" VARIANTS="base=X=1" bash scripts/r4_ab.sh || exit $?
TAG=s11c3bf REPS=1 ARGS="--dtype bf16" VARIANTS="base=X=1" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
