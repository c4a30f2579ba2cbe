#!/bin/bash
# round-5 GPU session 44: fp32 weight-gradient operands through a per-wave LDS-DMA ring
# (MEP_WG_DMA, variant wgdma) -- its parity (weight-gradient, cmu, ren, realformer tests), then the
# cfg3 / cfg5 / cfg2 / rfstate steps against the default build, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MEP_LIB=$PWD/variants/wgdma/libmep_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_cmu.py tests/test_gpu_ren.py tests/test_gpu_realformer.py tests/test_gpu_cfg5_shape.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t44.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t44.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t44.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in def wgdma; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    for c in cfg3 cfg5 cfg2 rfstate; do
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe --no-bf16 > gpurun_out/r5_b44_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b44_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b44_%s_%s.log'%(sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
k=d['kernels']
print('%-5s %-7s fp32 %.4f | wgrad %.1f | reduce %.1f' % (sys.argv[1], sys.argv[2], d['ms_per_step'], k['mep_wgrad']['avg_launch_us'], k.get('mep_reduce_grads', {}).get('avg_launch_us', 0)))
PY
    done
  done
done
echo ALLDONE
