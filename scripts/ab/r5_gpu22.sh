#!/bin/bash
# round-5 GPU session 22: mep_rfw_front (unify + projections per modality in one launch) -- kernel +
# realformer tests, then cfg2 / rfstate with MEP_RF_FRONT=1 / 0 and per-dispatch durations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rfw.py tests/test_gpu_realformer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t22.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t22.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t22.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    for c in cfg2 rfstate; do
      MEP_RF_FRONT=$v timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b22_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b22_${v}_$c.log; exit 1; }
      python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b22_%s_%s.log'%(sys.argv[1],sys.argv[2])).read().strip().splitlines()[-1])
print('front=%s'%sys.argv[1], sys.argv[2], d['ms_per_step'], {k: v['avg_launch_us'] for k, v in d['kernels'].items() if 'gemm' in k or 'front' in k})
PY
    done
  done
done
for cfg in cfg2 rfstate; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r5_do22_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/r5_do22_$cfg.log 2>&1; rc=$?
  echo "$cfg rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5_do22_$cfg.log; exit $rc; }
  python3 scripts/dispatch_order.py /tmp/r5_do22_$cfg > gpurun_out/r5_do22_$cfg.txt; head -4 gpurun_out/r5_do22_$cfg.txt; tail -1 gpurun_out/r5_do22_$cfg.txt
done
echo ALLDONE
