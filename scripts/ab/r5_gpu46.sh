#!/bin/bash
# round-5 GPU session 46: the fp32 epilogue forward with Wm staged behind each wave's first xp
# product (MEP_EPI_WM_LATE, variant late; the tile loop's first iteration peeled in both builds) --
# parity of both builds, then cfg3 / cfg5 against each other, three times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in def late; do
  lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
  MEP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_cmu.py tests/test_gpu_encoders.py tests/test_gpu_cfg5_shape.py tests/test_gpu_ren.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t46_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t46_$v.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t46_$v.log | head -20
  [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do
  for v in def late; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    for c in cfg3 cfg5; do
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe --no-bf16 > gpurun_out/r5_b46_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b46_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b46_%s_%s.log'%(sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
k=d['kernels']
print('%-5s %-5s fp32 %.4f | epi_fwd %.2f | epi_bwd %.1f' % (sys.argv[1], sys.argv[2], d['ms_per_step'], k['mep_block_epi_fwd']['avg_launch_us'], k['mep_block_epi_bwd']['avg_launch_us']))
PY
    done
  done
done
echo ALLDONE
