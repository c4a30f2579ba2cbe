#!/bin/bash
# round-4 GPU session 31: final tree -- GPU suite, smoke(), default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t31.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t31.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/t31.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke31.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke31.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default31.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default31.log | cut -c1-250
echo ALLDONE
