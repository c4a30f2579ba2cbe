#!/bin/bash
# round-4 GPU session 6: GPU suite, bench lines and a kernel trace of the cfg3 bf16 step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t6.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t6.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t6.log | head -20
[ $rc -eq 0 ] || exit $rc
TAG=s6 REPS=1 ARGS="--dtype bf16" VARIANTS="c3bf=X=1" bash scripts/r4_ab.sh || exit $?
TAG=s6f REPS=1 ARGS="--dtype fp32" VARIANTS="c3=X=1" bash scripts/r4_ab.sh || exit $?
TAG=s6c5 REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="c5bf=X=1" bash scripts/r4_ab.sh || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/s6prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dtype bf16 > gpurun_out/s6prof.log 2>&1 || exit $?
echo ALLDONE
