#!/bin/bash
# round-5 GPU session 48: the pooling forward with 24 time steps of loads per thread in flight (MEP_POOL_U) --
# engine tests, then cfg3 / cfg5 / rfstate against
# HEAD's build (variants/base), three times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cmu.py tests/test_gpu_ren.py tests/test_gpu_realformer.py tests/test_gpu_bf16.py tests/test_gpu_pool_fold.py tests/test_gpu_encoders.py tests/test_gpu_cfg5_shape.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t48.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t48.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t48.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in def base; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    for c in cfg3 cfg5 rfstate; do
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe --no-bf16 > gpurun_out/r5_b48_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b48_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b48_%s_%s.log'%(sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
k=d['kernels']
print('%-5s %-5s fp32 %.4f | pool %.2f' % (sys.argv[1], sys.argv[2], d['ms_per_step'], k['mep_pool_fwd']['avg_launch_us']))
PY
    done
  done
done
echo ALLDONE
