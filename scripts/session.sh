#!/bin/bash
# One GPU session on the box, by stages (replaces the per-session scripts of rounds 3-5):
#   TAG=r06_s1 STAGES="tests smoke bench" bash scripts/session.sh
# stages (run in the order given, each under its own time limit; the session stops at the first
# failure):
#   tests      pytest -m gpu (TESTS="tests/test_x.py ..." narrows it; default the whole suite;
#              KEEPGOING=1 runs past assertion failures)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py per workload of CFGS (default "cfg3"), BARGS appended
#   prof       rocprofv3 --kernel-trace --stats per workload (cfg3, cfg3_bf16, cfg5, ...)
#   traffic    the 32-B read-unit and WRITE_SIZE passes per workload (scripts/r4_counters.sh)
#   sq         the SQ counter groups per workload (scripts/r4_counters.sh)
#   ab         VARIANTS="name=-DFLAG=1;..." K=<launch>: variant builds timed by scripts/kbench.py
# outputs under gpurun_out/$TAG/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-session}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CFGS=${CFGS:-cfg3}
bargs() {
  case $1 in
    cfg3) echo "--config cfg3 --dtype fp32";; cfg3_bf16) echo "--config cfg3 --dtype bf16";;
    cfg2) echo "--config cfg2";; cfg5) echo "--config cfg5 --dtype fp32";; cfg5_bf16) echo "--config cfg5 --dtype bf16";;
    rfstate) echo "--config rfstate";; *) echo "unknown workload $1" >&2; exit 1;;
  esac; }
step() { local name=$1 limit=$2; shift 2
  echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  [ $rc -eq 0 ] || exit $rc; }
for s in ${STAGES:-tests smoke bench}; do
  case $s in
    tests)
      # KEEPGOING=1: the whole suite without -x, and later stages still run when the only failures
      # are test assertions (rc 1); any other status (a fault, an abort, a time limit) ends the session
      if [ "${KEEPGOING:-0}" = 1 ]; then
        echo "== tests"; timeout -k 10 ${TLIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 300 \
          --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
        echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -20
        [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
      else
        step tests ${TLIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread
        grep -E "passed|failed" $OUT/tests.log | tail -1
      fi;;
    smoke)
      step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')";;
    bench)
      for c in $CFGS; do
        step bench_$c 400 python3 bench.py $(bargs $c) $BARGS
        cp $OUT/bench_$c.log $OUT/bench_$c.json
      done;;
    prof)
      for c in $CFGS; do
        step prof_$c 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- \
          python3 bench.py --steps ${PSTEPS:-30} --warmup 5 --no-cpu-baseline --no-bf16 --no-probe $(bargs $c)
      done;;
    traffic|sq)
      OUT=$OUT/ctr STAGE=$s CFGS="$CFGS" PSTEPS=${PSTEPS:-20} bash scripts/r4_counters.sh || exit $?;;
    ab)
      step ab 900 bash scripts/ab.sh;;
    *) echo "unknown stage $s"; exit 1;;
  esac
done
echo SESSION_DONE
