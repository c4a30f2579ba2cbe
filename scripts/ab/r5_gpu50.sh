#!/bin/bash
# round-5 GPU session 50: the fp32 epilogues at D = 96 on 12 waves per workgroup (one tile per
# wave; <= 168 VGPRs, dropout paths out of line): variants w12 (forward + backward) and w12b
# (backward only) -- parity, then cfg3 against the default, three times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in w12 w12b; do
  MEP_LIB=$PWD/variants/$v/libmep_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_cmu.py tests/test_gpu_encoders.py tests/test_gpu_dp_exchange.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t50_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t50_$v.log | tail -2; grep -E "^FAILED|^ERROR|Error" gpurun_out/r5_t50_$v.log | head -20
  [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do
  for v in def w12 w12b; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-bf16 > gpurun_out/r5_b50_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b50_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b50_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
k=d['kernels']
print('%-5s cfg3 fp32 %.4f | epi_fwd %.2f | epi_bwd %.2f' % (sys.argv[1], d['ms_per_step'], k['mep_block_epi_fwd']['avg_launch_us'], k['mep_block_epi_bwd']['avg_launch_us']))
PY
  done
done
echo ALLDONE
