#!/bin/bash
# round-4 GPU session 3: SQ counter groups of every bench workload, then the bench lines (CPU
# baselines included)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGE=sq bash scripts/r4_counters.sh || exit $?
CPUB=10 bash scripts/bench_lines.sh || exit $?
echo ALLDONE
