#!/bin/bash
# round-4 GPU session 19 (re-run as the v4 set: 16-lane LayerNorm, weight-gradient rounds, fp32 DMA GEMM): GPU suite,
# smoke(); per workload the kernel trace + stats, the 32-B read units and WRITE_SIZE; the SQ groups
# of cfg5 bf16; then the bench lines of every config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -rf gpurun_out/r4ctr
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t19.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t19.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t19.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke19.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke19.log; [ $rc -eq 0 ] || exit $rc
STAGE=traffic PSTEPS=20 CFGS="cfg3_bf16 cfg3 cfg5_bf16 cfg5 cfg2" bash scripts/r4_counters.sh || exit $?
STAGE=sq CFGS="cfg5_bf16" bash scripts/r4_counters.sh || exit $?
echo ALLDONE
