#!/bin/bash
# round-5 GPU session 25: LDS layouts conflict-free under ds_read_b128's real lane groups (unify
# fp32 weight rows 16 KB + 8, SplitWS swizzle for odd pair counts) -- full GPU suite, bench lines
# for cfg3 (fp32 + bf16), cfg2, rfstate, then the SQ LDS-conflict counters of cfg3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t25.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t25.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t25.log | head -20
[ $rc -eq 0 ] || exit $rc
for c in cfg3 cfg2 rfstate; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b25_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b25_$c.log; exit 1; }
  python3 - $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b25_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
b=d.get('bf16') or {}
f=lambda x: ' '.join('%s %.1f'%(n.replace('mep_',''), v['avg_launch_us']) for n, v in sorted(x.items(), key=lambda kv: -kv[1]['ms_per_step'])[:8])
print(sys.argv[1], 'fp32', d['ms_per_step'], f(d['kernels']))
if b: print(sys.argv[1], 'bf16', b['ms_per_step'], f(b['kernels']))
PY
done
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --kernel-trace -d /tmp/r5_c25 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r5_c25.log 2>&1; echo "ctr rc=$?"
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob('/tmp/r5_c25/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('(anonymous namespace)::', '')[:40]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(acc.items()):
    if v.get('SQ_LDS_IDX_ACTIVE'):
        print('%-40s conflict share %.3f' % (k, v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']))
PY
echo ALLDONE
