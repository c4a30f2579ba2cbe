#!/bin/bash
# round-5 GPU session 45: clip + Adam with the thread's first float4 loaded before the norm's
# partial sums (one memory latency instead of two) -- engine tests, then cfg3 / cfg2 / cfg5 against
# HEAD's build (variants/base), three times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cmu.py tests/test_gpu_ren.py tests/test_gpu_realformer.py tests/test_gpu_dp.py tests/test_gpu_dp_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t45.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t45.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t45.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in def base; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    for c in cfg3 cfg2 cfg5; do
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe --no-bf16 > gpurun_out/r5_b45_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b45_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b45_%s_%s.log'%(sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
k=d['kernels']
print('%-5s %-5s fp32 %.4f | adam %.2f | reduce %.1f' % (sys.argv[1], sys.argv[2], d['ms_per_step'], k['mep_clip_adam_ext']['avg_launch_us'], k.get('mep_reduce_grads', {}).get('avg_launch_us', 0)))
PY
    done
  done
done
echo ALLDONE
