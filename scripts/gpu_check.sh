#!/bin/bash
# GPU-box session: tests, smoke, short bench.  Stops at the first GPU fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139|-6|-11) return 0;; *) return 1;; esac; }
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name -- stopping"; exit $rc; fi
  return $rc
}
STEPS="${STEPS:-pytest smoke bench}"
for s in $STEPS; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 600 python bench.py --steps ${BSTEPS:-100} --warmup 10 --cpu-budget ${CPUB:-8} ;;
    prof)   step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline ;;
  esac
done
exit 0
