#!/bin/bash
# GPU-box inner loop: gpu tests (stop on failure), then per-kernel timings of the bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu ${PYTEST_X--x} -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pt.log 2>&1
rc=$?; tail -n 30 gpurun_out/pt.log | grep -v "amdgpu.ids"; echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
true
[ -n "$BENCH" ] && timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids
exit $rc
