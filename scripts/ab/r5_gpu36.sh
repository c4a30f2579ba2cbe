#!/bin/bash
# round-5 GPU session 36: mep_wgemm_sum tile shapes (16 x 16 NI columns, GP k pairs per load group:
# default NI 1 / GP 6 against the variants) and the unfused launches, cfg2, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rfw.py -m gpu -x -q -k "sum" --timeout 120 --timeout-method thread > gpurun_out/r5_t36.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t36.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t36.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in def s14 s24 s28 off; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    on=1; [ $v = off ] && on=0
    MEP_LIB=$lib MEP_RF_WGEMM_SUM=$on timeout -k 10 300 python3 bench.py --config cfg2 --no-cpu-baseline --no-probe > gpurun_out/r5_b36_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b36_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b36_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('kernels', {})
print('%s %.4f ms  %s' % (sys.argv[1], d['ms_per_step'], {n: v.get('avg_launch_us') for n, v in k.items() if 'sum' in n or 'wgemm' in n}))
PY
  done
done
echo ALLDONE
