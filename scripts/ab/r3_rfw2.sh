#!/bin/bash
# realformer tests, then kernel traces of cfg2 (base, timing-only variants)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_realformer.py tests/test_gpu_encoders.py tests/test_gpu_robot.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_rf.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/pt_rf.log | tail -n 15; echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
V="${V:-base now}" BARGS="--config cfg2" bash scripts/r3_vtrace.sh
