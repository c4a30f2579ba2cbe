#!/bin/bash
# rocprofv3 passes for one bench workload: kernel trace + stats, then separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (TCC slots cannot hold both; never combined with other tracing).
#   TAG=cfg5_bf16 BARGS="--config cfg5 --dtype bf16" bash scripts/profile.sh
# -> gpurun_out/prof_<TAG>/{trace,fetch,write}; summarise with
#   python scripts/parse_prof.py r03_vN_<...> gpurun_out/prof_<TAG>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-cfg3}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps ${PSTEPS:-30} --warmup 5 --no-cpu-baseline $BARGS"
run() { local name=$1; shift
  echo "== $TAG $name"; timeout -k 10 600 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -1 $OUT/$name.log
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
run trace rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS
run fetch rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS
run write rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS
