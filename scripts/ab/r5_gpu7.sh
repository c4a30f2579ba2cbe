#!/bin/bash
# round-5 GPU session 7: bench with stamp-kernel launch timing + rocprofv3 of the same command;
# State_Transfer at the reference configuration (rf_state_ref)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_realformer.py -x -v -s --timeout 120 --timeout-method thread -k "state" > gpurun_out/r5_t7.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|worst|PASS|FAIL" gpurun_out/r5_t7.log | tail -12; grep -E "^E " gpurun_out/r5_t7.log | head -10
timeout -k 10 300 python3 bench.py > gpurun_out/r5_bench7.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r5_bench7.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof7 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r5_bench7_prof.log 2>&1; rc=$?; echo "prof rc=$rc"
python3 scripts/cmp_prof.py gpurun_out/r5_bench7_prof.log gpurun_out/r5_prof7
echo ALLDONE
timeout -k 10 300 python3 bench.py --config rfstate > gpurun_out/r5_bench7_rfstate.log 2>&1; rc=$?; echo "rfstate bench rc=$rc"; tail -c 800 gpurun_out/r5_bench7_rfstate.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof7_rfstate -o run --output-format csv -- python3 bench.py --config rfstate --no-cpu-baseline > gpurun_out/r5_bench7_rfstate_prof.log 2>&1; rc=$?; echo "rfstate prof rc=$rc"
echo ALLDONE2
