#!/bin/bash
# round-4 GPU session 14: smoke(), the default bench line, A/B of the long-forward chunk prefetch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke14.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke14.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default14.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default14.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
TAG=s14c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="base=X=1;cpf=MEP_LIB=variants/cpf/libmep_hip.so" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
