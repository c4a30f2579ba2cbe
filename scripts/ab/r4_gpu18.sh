#!/bin/bash
# round-4 GPU session 18: ren dropout norm-fold test (current vs previous LayerNorm kernels);
# wide-backward staging ring depth A/B (cfg5 bf16 / fp32)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=tests/test_gpu_rccl.py::test_norm_fold_matches_optimizer_norm_pass_ren_dropout
for v in new new old old; do
  if [ $v = old ]; then export MEP_LIB=$PWD/variants/old/libmep_hip.so; else unset MEP_LIB; fi
  timeout -k 10 180 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/t18_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep -E "AssertionError|passed|failed" gpurun_out/t18_$v.log | head -3
  [ $rc -le 1 ] || exit $rc
done
unset MEP_LIB
V="base=X=1;ns3=MEP_LIB=$PWD/variants/ns3/libmep_hip.so;ns4=MEP_LIB=$PWD/variants/ns4/libmep_hip.so"
TAG=s18c5bf REPS=2 STEPS=30 ARGS="--config cfg5 --dtype bf16" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
TAG=s18c5 REPS=1 STEPS=30 ARGS="--config cfg5 --dtype fp32" VARIANTS="$V" bash scripts/r4_ab.sh || exit $?
echo ALLDONE
