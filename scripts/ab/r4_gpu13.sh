#!/bin/bash
# round-4 GPU session 13: GPU suite, SQ counter groups of every workload, then the bench lines (CPU baselines)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t13.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t13.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t13.log | head -20
[ $rc -eq 0 ] || exit $rc
STAGE=sq CFGS="${CFGS:-cfg3_bf16 cfg3 cfg5_bf16 cfg5 cfg2}" bash scripts/r4_counters.sh || exit $?
CPUB=10 bash scripts/bench_lines.sh || exit $?
echo ALLDONE
