#!/bin/bash
# rocprofv3 kernel-trace stats of one bench workload: BARGS="--config cfg2" TAG=cfg2 bash scripts/r3_trace.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-cfg2}
OUT=gpurun_out/tr_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline $BARGS > $OUT/log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $OUT/log | cut -c1-300
f=$(find $OUT -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print('%-70s %5s %10.1f' % (r['Name'].replace('(anonymous namespace)::', '')[:70], r['Calls'], float(r['AverageNs']) / 1e3))
PY
exit $rc
