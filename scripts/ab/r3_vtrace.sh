#!/bin/bash
# rocprofv3 kernel averages of one workload per variant build: V="base now rot4" BARGS="--config cfg2" bash scripts/r3_vtrace.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${V:-base}; do
  OUT=gpurun_out/vt_$v; rm -rf $OUT; mkdir -p $OUT
  lib=""; [ "$v" != base ] && lib=variants/$v/libmep_hip.so
  MEP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline $BARGS > $OUT/log 2>&1
  rc=$?
  f=$(find $OUT -name '*kernel_stats.csv' | head -1)
  echo "== $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/log)"
  python3 - "$f" "${K:-k_wgemm|k_rfw|k_wsplit}" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name'].replace('(anonymous namespace)::', '')
    if re.search(sys.argv[2], n):
        print('   %-60s %5s %8.1f' % (n[:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
  case $rc in 0) ;; *) exit $rc;; esac
done
