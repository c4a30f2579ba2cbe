#!/bin/bash
# full GPU suite + smoke, then the wgrad kernel of every workload (both precisions)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS="pytest smoke" bash scripts/gpu_check.sh || exit $?
for cfg in "" "--dtype bf16" "--config cfg5" "--config cfg5 --dtype bf16" "--config cfg2"; do
  echo "#### $cfg"
  K="k_wgrad" V="base" BARGS="$cfg" bash scripts/r3_vtrace.sh || exit $?
done
