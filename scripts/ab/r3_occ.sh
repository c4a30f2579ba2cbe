#!/bin/bash
# k_wgrad at two workgroups per CU (variants/occ2): parity tests through the variant, then kernel
# traces and bench lines against the base build on the same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MEP_LIB=variants/occ2/libmep_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_cmu.py tests/test_gpu_ren.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/occ_tests.log 2>&1
rc=$?; tail -3 gpurun_out/occ_tests.log; [ $rc = 0 ] || exit $rc
for cfg in "" "--config cfg5" "--config cfg2"; do
  echo "#### $cfg"
  K="k_wgrad|k_reduce" V="base occ2" BARGS="$cfg" bash scripts/r3_vtrace.sh || exit $?
done
