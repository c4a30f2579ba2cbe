#!/bin/bash
# round-5 GPU session 6: GPU suite (new cfg5 bench-shape, tgemm N%32 tests), then the bench with
# hipExtLaunchKernel launch timing and the rocprofv3 stats of the same command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > gpurun_out/r5_bench6.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1200 gpurun_out/r5_bench6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof6 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r5_bench6_prof.log 2>&1; rc=$?; echo "prof rc=$rc"
python3 scripts/cmp_prof.py gpurun_out/r5_bench6_prof.log gpurun_out/r5_prof6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "not rf_state_ref" > gpurun_out/r5_t6.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t6.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t6.log | head -20
echo ALLDONE
