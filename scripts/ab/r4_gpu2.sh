#!/bin/bash
# round-4 GPU session 2: full GPU suite, bench lines (cfg3 fp32 / bf16, cfg5 bf16)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" gpurun_out/t2.log | tail -3; grep -E "^FAILED|^ERROR" gpurun_out/t2.log | head -30
grep -E "^bf16|worst tensors" gpurun_out/t2.log | head -40
TAG=lines REPS=1 VARIANTS="cfg3=X=1" ARGS="--dtype fp32" bash scripts/r4_ab.sh || exit $?
TAG=lines_bf REPS=1 VARIANTS="cfg3bf=X=1" ARGS="--dtype bf16" bash scripts/r4_ab.sh || exit $?
TAG=lines_c5bf REPS=1 VARIANTS="cfg5bf=X=1" ARGS="--config cfg5 --dtype bf16" bash scripts/r4_ab.sh || exit $?
mkdir -p gpurun_out/r4ctr && timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_sum --kernel-trace -d gpurun_out/r4ctr/cal_req2 -o run --output-format csv -- ./scripts/micro/fetch_cal > gpurun_out/cal_req2.log 2>&1 || exit $?
echo cal_req2 ok
[ "${TRAFFIC:-1}" = 1 ] && { STAGE=traffic PSTEPS=20 bash scripts/r4_counters.sh || exit $?; }
echo ALLDONE
