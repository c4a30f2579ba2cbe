#!/bin/bash
# round-5 GPU session 11: key-pair dS transpose writes (MEP_BWD_TPAIR) -- attention / model suites,
# then cfg3 and cfg5 A/B against the 16-bit writes (variants/notpair)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t11.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t11.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t11.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in main notpair; do
    if [ $v = main ]; then L=""; else L=variants/$v/libmep_hip.so; fi
    for c in cfg3 cfg5; do
    MEP_LIB=$L timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-probe > gpurun_out/r5_b11_${v}_$c.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5_b11_${v}_$c.log; exit 1; }
    python3 - $v $c <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b11_%s_%s.log'%(sys.argv[1],sys.argv[2])).read().strip().splitlines()[-1])
k=d['kernels']; b=d['bf16']['kernels']
print(sys.argv[1], sys.argv[2], 'fp32', d['ms_per_step'], 'bwd', k['mep_attn_bwd']['avg_launch_us'], '| bf16', d['bf16']['ms_per_step'], 'bwd', b['mep_attn_bwd']['avg_launch_us'])
PY
    done
  done
done
echo ALLDONE
