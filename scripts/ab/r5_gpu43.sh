#!/bin/bash
# round-5 GPU session 43: the 16-lane DPP sums as fused v_add_f32_dpp steps, paired (MEP_ROW16_FUSED) --
# the epilogue / LayerNorm tests, then cfg3 / cfg5 against HEAD's build (variants/base), twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_pool_fold.py tests/test_gpu_cmu.py tests/test_gpu_encoders.py tests/test_gpu_ren.py tests/test_gpu_cfg5_shape.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t43.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t43.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t43.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in def base; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    for c in cfg3 cfg5; do
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b43_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b43_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b43_%s_%s.log'%(sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
b=d.get('bf16')
top=lambda x: ' '.join('%s %.1f' % (n.replace('mep_', ''), v['avg_launch_us']) for n, v in sorted(x['kernels'].items(), key=lambda kv: -kv[1]['ms_per_step'])[:6])
print('%-5s %s fp32 %.4f | %s' % (sys.argv[1], sys.argv[2], d['ms_per_step'], top(d)))
if b: print('%-5s %s bf16 %.4f | %s' % (sys.argv[1], sys.argv[2], b['ms_per_step'], top(b)))
PY
    done
  done
done
echo ALLDONE
