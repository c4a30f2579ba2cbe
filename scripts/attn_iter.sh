#!/bin/bash
# GPU-box inner loop for the attention kernels: attention / model parity tests, then per-kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pt.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/pt.log | tail -15; echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 150 python scripts/kbench.py --reps 50 ${KB_ARGS} 2>&1 | grep -v amdgpu.ids
