#!/bin/bash
# round-5 GPU session 38: per-workgroup phase trace of the fp32 epilogue forward (epi_fwd_wp2r),
# including wave 0's second tile (stamps 6 / 7)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
MEP_LIB=$PWD/variants/etrace/libmep_hip.so timeout -k 10 300 python3 scripts/epi_trace1.py > gpurun_out/r5_trace38.log 2>&1; rc=$?
cat gpurun_out/r5_trace38.log | tail -30
exit $rc
