#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_X=" " bash scripts/quick.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
WORKLOADS="cfg3:;cfg3_bf16:--dtype bf16;cfg5:--config cfg5" SKIP_BENCH=1 bash scripts/r3_prof.sh
