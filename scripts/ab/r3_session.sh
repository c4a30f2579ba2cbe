#!/bin/bash
# Round-3 GPU session: MFMA rate micro-benchmark, GPU tests, A/B of attention variants, bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -x scripts/micro/mfma_rate ] && [ -z "$SKIP_MICRO" ]; then
  timeout -k 10 60 scripts/micro/mfma_rate > gpurun_out/mfma_rate.log 2>&1; rc=$?; cat gpurun_out/mfma_rate.log
  case $rc in 124|134|137|139) exit $rc;; esac
fi
if [ -z "$SKIP_TESTS" ]; then
  bash scripts/quick.sh; rc=$?
  case $rc in 124|134|137|139) exit $rc;; esac
fi
[ -n "$SKIP_AB" ] || bash scripts/r3_ab.sh || exit $?
[ -n "$SKIP_BENCH" ] || bash scripts/bench_lines.sh
