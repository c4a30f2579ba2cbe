#!/bin/bash
# round-5 GPU session 9: default bench line (single-phase fp32 epilogue forward) + rocprofv3 of the
# same command; cfg5 and rfstate lines with their rocprofv3 stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > gpurun_out/r5_bench9.log 2>&1; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || { tail -5 gpurun_out/r5_bench9.log; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof9 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r5_bench9_prof.log 2>&1; rc=$?; echo "prof rc=$rc"
python3 scripts/cmp_prof.py gpurun_out/r5_bench9_prof.log gpurun_out/r5_prof9
[ $rc -eq 0 ] || exit $rc
for c in cfg5 rfstate cfg2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof9_$c -o run --output-format csv -- python3 bench.py --config $c > gpurun_out/r5_bench9_$c.log 2>&1; rc=$?; echo "$c rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r5_bench9_$c.log; exit $rc; }
  python3 scripts/cmp_prof.py gpurun_out/r5_bench9_$c.log gpurun_out/r5_prof9_$c
done
echo ALLDONE
