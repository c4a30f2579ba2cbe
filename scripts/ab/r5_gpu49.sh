#!/bin/bash
# round-5 GPU session 49: the attention forward's V^T operand from V row loads (8 bytes bf16 /
# 16 bytes fp32, the fp32 rows split into their 3 parts in row layout) transposed through LDS
# (ds_read_b64_tr_b16; MEP_FWD_VTR + MEP_FWD_VTR32, variant vtr2) instead of 16 per-element
# gathers per key chunk -- parity, then cfg3 / cfg5 (fp32 + nested bf16) against the default, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MEP_LIB=$PWD/variants/vtr2/libmep_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_cfg5_shape.py tests/test_gpu_pool_fold.py tests/test_gpu_encoders.py tests/test_gpu_cmu.py tests/test_gpu_ren.py tests/test_gpu_realformer.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t49.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t49.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t49.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in def vtr2; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    for c in cfg3 cfg5; do
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b49_${v}_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b49_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b49_%s_%s.log'%(sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
for tag, x in (('fp32', d), ('bf16', d['bf16'])):
    k=x['kernels']
    print('%-5s %-5s %s %.4f | attn_fwd %.1f | attn_bwd %.1f' % (sys.argv[1], sys.argv[2], tag, x['ms_per_step'], k['mep_attn_fwd']['avg_launch_us'], k['mep_attn_bwd']['avg_launch_us']))
PY
    done
  done
done
echo ALLDONE
