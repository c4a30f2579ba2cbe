#!/bin/bash
# round-4 GPU session 12: profile set v2 -- per workload the kernel trace + stats, the 32-B read
# units and WRITE_SIZE (scripts/r4_traffic.py), then the SQ groups (scripts/r4_ctr_summary.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -rf gpurun_out/r4ctr
STAGE=traffic PSTEPS=20 CFGS="${CFGS:-cfg3_bf16 cfg3 cfg5_bf16 cfg5 cfg2}" bash scripts/r4_counters.sh || exit $?
echo ALLDONE
