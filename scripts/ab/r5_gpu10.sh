#!/bin/bash
# round-5 GPU session 10: head quads for the Tk > 64 attention kernels -- Ren-MME / bf16 / cfg5
# suites, then the cfg5 A/B against head pairs (variants/noquad)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ren.py tests/test_gpu_bf16.py tests/test_gpu_cfg5_shape.py tests/test_gpu_cmu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t10.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t10.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t10.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in main noquad; do
    if [ $v = main ]; then L=""; else L=variants/$v/libmep_hip.so; fi
    MEP_LIB=$L timeout -k 10 300 python3 bench.py --config cfg5 --no-cpu-baseline --no-probe > gpurun_out/r5_b10_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5_b10_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b10_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
k=d['kernels']; b=d['bf16']['kernels']
print(sys.argv[1], 'fp32', d['ms_per_step'], 'fwd', k['mep_attn_fwd']['avg_launch_us'], 'bwd', k['mep_attn_bwd']['avg_launch_us'],
      '| bf16', d['bf16']['ms_per_step'], 'fwd', b['mep_attn_fwd']['avg_launch_us'], 'bwd', b['mep_attn_bwd']['avg_launch_us'])
PY
  done
done
echo ALLDONE
