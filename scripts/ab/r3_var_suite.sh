#!/bin/bash
# GPU suite on a variant build (no -x), then kernel traces: VAR=wm2 K='k_epi' BARGS='' V='base wm2' bash scripts/r3_var_suite.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MEP_LIB=variants/$VAR/libmep_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pt_$VAR.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/pt_$VAR.log | grep -v amdgpu.ids | tail -n 25; echo "pytest($VAR) rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/r3_vtrace.sh
