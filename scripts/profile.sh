#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (TCC slots cannot hold both; never combined with other tracing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--steps ${PSTEPS:-30} --warmup 5 --no-cpu-baseline"
run() { local name=$1; shift
  echo "== $name"; timeout -k 10 600 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $OUT/$name.log
  case $rc in 124|134|137|139) echo FATAL; exit $rc;; esac; }
run trace rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS
run fetch rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS
run write rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS
find $OUT -name "*.csv" | head -20
