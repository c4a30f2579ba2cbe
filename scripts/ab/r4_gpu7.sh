#!/bin/bash
# round-4 GPU session 7: GPU suite; A/B of the bf16 backward-attention changes (variants/hd = the
# previous commit's library); parity and A/B of the single-phase fp32 forward epilogue (variants/wm2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t7.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t7.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t7.log | head -20
[ $rc -eq 0 ] || exit $rc
TAG=s7c3bf REPS=2 ARGS="--dtype bf16" VARIANTS="base=X=1;hd=MEP_LIB=variants/hd/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
TAG=s7c5bf REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="base=X=1;hd=MEP_LIB=variants/hd/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
MEP_LIB=variants/wm2/libmep_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_cmu.py tests/test_gpu_ren.py tests/test_gpu_encoders.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t7wm2.log 2>&1
echo "wm2 pytest rc=$?"; grep -E "passed|failed" gpurun_out/t7wm2.log | tail -2; grep -E "^FAILED|^E  " gpurun_out/t7wm2.log | head -20
TAG=s7c3 REPS=2 ARGS="--dtype fp32" VARIANTS="base=X=1;wm2=MEP_LIB=variants/wm2/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
