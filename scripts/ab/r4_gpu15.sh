#!/bin/bash
# round-4 GPU session 15: GPU suite; smoke(); the default bench line; A/B of the fusable DPP
# reductions against HEAD (variants/hd) and of the long-forward chunk prefetch (variants/cpf)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t15.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t15.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t15.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke15.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke15.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default15.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default15.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
TAG=s15c3bf REPS=2 ARGS="--dtype bf16" VARIANTS="base=X=1;hd=MEP_LIB=variants/hd/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
TAG=s15c5bf REPS=1 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="base=X=1;hd=MEP_LIB=variants/hd/libmep_hip.so;cpf=MEP_LIB=variants/cpf/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
