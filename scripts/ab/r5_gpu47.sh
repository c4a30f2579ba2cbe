#!/bin/bash
# round-5 GPU session 47: the final tree -- the whole GPU suite, smoke(), and the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_t47.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t47.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/r5_t47.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke47.log 2>&1; rc=$?; tail -2 gpurun_out/r5_smoke47.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/r5_bench47.json 2> gpurun_out/r5_bench47.err || { tail -5 gpurun_out/r5_bench47.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r5_bench47.json').read().strip().splitlines()[-1])
print(d['metric'], d['value'], d['unit'], d['ms_per_step'], d['dtype'], 'bf16', d['bf16']['value'], d['bf16']['ms_per_step'])
print('roofline', d['roofline']['kernel'], d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])
print('sum kernels', round(sum(v['ms_per_step'] for v in d['kernels'].values()), 4))
PY
echo ALLDONE
