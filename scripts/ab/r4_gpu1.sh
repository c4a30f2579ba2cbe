#!/bin/bash
# round-4 GPU session 1: GPU suite, FETCH calibration, cfg5 A/B (head pairs, XCD packing), bf16 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" gpurun_out/t1.log | tail -3; grep -E "^FAILED|^ERROR" gpurun_out/t1.log | head -30
STAGE=cal bash scripts/r4_counters.sh || exit $?
TAG=cfg5 ARGS="--config cfg5 --dtype fp32" REPS=2 VARIANTS="base=X=1;nohp=MEP_LIB=variants/nohp/libmep_hip.so;noxcd=MEP_WG_XCD=0" bash scripts/r4_ab.sh || exit $?
TAG=bf16 REPS=1 VARIANTS="cfg3bf=X=1" ARGS="--dtype bf16" bash scripts/r4_ab.sh || exit $?
TAG=bf16c5 REPS=1 VARIANTS="cfg5bf=X=1" ARGS="--config cfg5 --dtype bf16" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
