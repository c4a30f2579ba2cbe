#!/bin/bash
# rocprofv3 kernel stats + FETCH/WRITE PMC passes of every bench workload (scripts/profile.sh),
# then the bench lines.  Stops at the first fatal status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WL=("cfg3:" "cfg3_bf16:--dtype bf16" "cfg5:--config cfg5" "cfg5_bf16:--config cfg5 --dtype bf16" "cfg2:--config cfg2")
[ -n "$WORKLOADS" ] && IFS=';' read -ra WL <<< "$WORKLOADS"
for w in "${WL[@]}"; do
  tag=${w%%:*}; args=${w#*:}
  TAG=$tag BARGS="$args" PSTEPS=${PSTEPS:-20} bash scripts/profile.sh || exit $?
done
[ -n "$SKIP_BENCH" ] || bash scripts/bench_lines.sh
