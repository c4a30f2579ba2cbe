#!/bin/bash
# k_wgrad launch size A/B (MEP_WG_TARGET workgroups), cfg3 and cfg2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "" "--config cfg2"; do for t in 512 384 768 1024; do
  echo "#### $cfg target=$t"
  MEP_WG_TARGET=$t K="k_wgrad|k_reduce" V=base BARGS="$cfg" bash scripts/r3_vtrace.sh || exit $?
done; done
