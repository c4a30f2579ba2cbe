#!/bin/bash
# round-5 GPU session 30: full GPU suite (XCD-ordered unify tasks, epilogue XCD order, ABI 4), unify
# XCD order A/B, and the epilogues launched twice per step (second launch on a warm L2) from a
# kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_t30.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r5_t30.log | tail -2; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_t30.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    MEP_UNIFY_XCD=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/r5_b30_$v.log 2>&1 || { echo "bench failed"; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b30_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
print('unify_xcd=%s fp32 %.4f unify %.1f | bf16 %.4f unify %.1f' % (sys.argv[1], d['ms_per_step'], d['kernels']['mep_unify']['avg_launch_us'], d['bf16']['ms_per_step'], d['bf16']['kernels']['mep_unify']['avg_launch_us']))
PY
  done
done
for dt in fp32 bf16; do
  MEP_DEV_EPI_TWICE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r5_do30_$dt -o run --output-format csv -- python3 bench.py --config cfg3 --dtype $dt --no-bf16 --steps 8 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/r5_do30_$dt.log 2>&1; rc=$?
  echo "$dt rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5_do30_$dt.log; exit $rc; }
  python3 scripts/dispatch_order.py /tmp/r5_do30_$dt k_unify | tee gpurun_out/r5_do30_$dt.txt
done
echo ALLDONE
