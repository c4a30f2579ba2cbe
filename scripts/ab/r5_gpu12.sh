#!/bin/bash
# round-5 GPU session 12: 2-part fp32 weight gradients (variants/wg2, MEP_WG_PARTS=2): GPU suite on
# the variant, then the cfg3 / cfg5 A/B against the 3-part build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MEP_LIB=variants/wg2/libmep_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_t12.log 2>&1
rc=$?; echo "pytest(wg2) rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t12.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/r5_t12.log | head -30
for rep in 1 2; do
  for v in main wg2; do
    if [ $v = main ]; then L=""; else L=variants/$v/libmep_hip.so; fi
    for c in cfg3 cfg5; do
    MEP_LIB=$L timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe --no-bf16 > gpurun_out/r5_b12_${v}_$c.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5_b12_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b12_%s_%s.log'%(sys.argv[1],sys.argv[2])).read().strip().splitlines()[-1])
k=d['kernels']
print(sys.argv[1], sys.argv[2], 'fp32', d['ms_per_step'], 'wgrad', k['mep_wgrad']['avg_launch_us'])
PY
    done
  done
done
echo ALLDONE
