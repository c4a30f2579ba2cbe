#!/bin/bash
# round-4 GPU session 13: SQ counter groups of every workload, then the bench lines (CPU baselines)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGE=sq CFGS="${CFGS:-cfg3_bf16 cfg3 cfg5_bf16 cfg5 cfg2}" bash scripts/r4_counters.sh || exit $?
CPUB=10 bash scripts/bench_lines.sh || exit $?
echo ALLDONE
