#!/bin/bash
# k_sum_rows on the source count + the cfg2 norm fold: tests, traces, bench lines (same box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sumfold.py tests/test_gpu_cmu.py tests/test_gpu_ren.py tests/test_gpu_realformer.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc = 0 ] || exit $rc
for cfg in "" "--config cfg5" "--config cfg2"; do
  echo "#### $cfg"
  K="k_sum_rows|k_sqnorm|k_clip|k_reduce" V="base" BARGS="$cfg" bash scripts/r3_vtrace.sh || exit $?
done
for i in 1 2; do for f in 1 0; do
  MEP_NORM_FOLD=$f timeout -k 10 120 python3 bench.py --config cfg2 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit $?
  echo "bench cfg2 norm=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json) $(grep -o '"loss": [-0-9.e]*' gpurun_out/ab.json)"
done; done
