#!/bin/bash
# round-5 GPU session 5: bench with in-step launch timing; rocprofv3 stats (csv) of the same command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > gpurun_out/r5_bench5.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r5_bench5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r5_bench5_prof.log 2>&1; rc=$?; echo "prof rc=$rc"
python3 scripts/cmp_prof.py gpurun_out/r5_bench5_prof.log gpurun_out/r5_prof5
echo ALLDONE
