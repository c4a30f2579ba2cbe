#!/bin/bash
# round-4 GPU session 16: GPU suite (32-bit dropout hash, regenerated dropout fixtures); A/B against
# HEAD (variants/hd: the 64-bit hash) and of the transposed-dS backward (variants/tr)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t16.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t16.log | head -20
[ $rc -eq 0 ] || exit $rc
TAG=s16c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="base=X=1;hd=MEP_LIB=variants/hd/libmep_hip.so;tr=MEP_LIB=variants/tr/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
TAG=s16c5 REPS=1 STEPS=20 ARGS="--config cfg5 --dtype fp32" VARIANTS="base=X=1;hd=MEP_LIB=variants/hd/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
TAG=s16c3bf REPS=1 ARGS="--dtype bf16" VARIANTS="base=X=1;tr=MEP_LIB=variants/tr/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
