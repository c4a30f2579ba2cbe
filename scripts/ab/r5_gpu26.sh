#!/bin/bash
# round-5 GPU session 26: the per-dispatch sequence of a cfg3 step (fp32 and bf16), torch kernels
# included, and the LDS-conflict share per kernel after the layout fixes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for dt in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r5_do26_$dt -o run --output-format csv -- python3 bench.py --config cfg3 --dtype $dt --no-bf16 --steps 8 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/r5_do26_$dt.log 2>&1; rc=$?
  echo "$dt rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5_do26_$dt.log; exit $rc; }
  python3 scripts/dispatch_order.py /tmp/r5_do26_$dt k_unify | tee gpurun_out/r5_do26_$dt.txt
done
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --kernel-trace -d /tmp/r5_c26 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r5_c26.log 2>&1; echo "ctr rc=$?"
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('/tmp/r5_c26/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:48]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(acc.items()):
    if v.get('SQ_LDS_IDX_ACTIVE'):
        print('%-48s conflict share %.3f' % (k, v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']))
PY
echo ALLDONE
