#!/bin/bash
# round-5 GPU session 51: the epilogue products' fragment ring depth (MEP_TG_RING 1 / 3 against the
# default 2) now that the bf16 epilogues run 12 waves per workgroup -- cfg3 fp32 + nested bf16, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MEP_LIB=$PWD/variants/ring3/libmep_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_cmu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t51.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t51.log | tail -2
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in def ring1 ring3; do
    lib=""; [ -f variants/$v/libmep_hip.so ] && lib=$PWD/variants/$v/libmep_hip.so
    MEP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/r5_b51_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b51_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b51_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
for tag, x in (('fp32', d), ('bf16', d['bf16'])):
    k=x['kernels']
    print('%-5s %s %.4f | epi_fwd %.2f | epi_bwd %.2f' % (sys.argv[1], tag, x['ms_per_step'], k['mep_block_epi_fwd']['avg_launch_us'], k['mep_block_epi_bwd']['avg_launch_us']))
PY
  done
done
echo ALLDONE
