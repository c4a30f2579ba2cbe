#!/bin/bash
# round-5 GPU session 1: the new bench line (fp32 headline + nested bf16, graph-replay kernel
# times, measured HBM peak) and the rocprofv3 stats of the same command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > gpurun_out/r5_bench1.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r5_bench1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof1 -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/r5_bench1_prof.log 2>&1; rc=$?; echo "prof rc=$rc"
find gpurun_out/r5_prof1 -name "*stats*" | head
echo ALLDONE
