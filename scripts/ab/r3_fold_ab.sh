#!/bin/bash
# folded sums / folded norm: GPU tests, then kernel traces and bench lines, fold on / off, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sumfold.py tests/test_gpu_cmu.py tests/test_gpu_ren.py tests/test_gpu_rccl.py tests/test_gpu_pool_fold.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc = 0 ] || exit $rc
for cfg in "" "--config cfg5"; do
  for f in "1 1" "0 1" "1 0"; do
    set -- $f
    echo "#### MEP_SUM_FOLD=$1 MEP_NORM_FOLD=$2 $cfg"
    MEP_SUM_FOLD=$1 MEP_NORM_FOLD=$2 K="k_clip|k_sqnorm|k_reduce|k_attn_bwd|k_sum_rows" V="base" BARGS="$cfg" bash scripts/r3_vtrace.sh || exit $?
  done
done
for i in 1 2; do for f in "1 1" "0 1" "1 0"; do
  set -- $f
  MEP_SUM_FOLD=$1 MEP_NORM_FOLD=$2 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit $?
  echo "bench cfg3 sum=$1 norm=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
done; done
