#!/bin/bash
# round-5 GPU session 15: realformer epilogue forward for large launches at 3 waves per SIMD (two
# tiles per CU) -- realformer suite, then rfstate / cfg2 A/B against the default kernel only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_realformer.py tests/test_gpu_rfw.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t15.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t15.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t15.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in main nobig; do
    if [ $v = main ]; then L=""; else L=variants/$v/libmep_hip.so; fi
    for c in rfstate cfg2; do
    MEP_LIB=$L timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b15_${v}_$c.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5_b15_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b15_%s_%s.log'%(sys.argv[1],sys.argv[2])).read().strip().splitlines()[-1])
k=d['kernels']
print(sys.argv[1], sys.argv[2], d['ms_per_step'], 'fwd', k['mep_rfw_epi_fwd']['avg_launch_us'], 'bwd', k['mep_rfw_epi_bwd']['avg_launch_us'])
PY
    done
  done
done
echo ALLDONE
