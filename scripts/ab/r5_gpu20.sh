#!/bin/bash
# round-5 GPU session 20: mep_wgemm_ws with guard-free products, a fragment ring and batched
# weight copies -- kernel + realformer tests, bench A/B, per-dispatch durations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/ab/r5_gpu18.sh || exit $?
export TMPDIR=/tmp
for cfg in cfg2 rfstate; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r5_do20_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/r5_do20_$cfg.log 2>&1; rc=$?
  echo "$cfg rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5_do20_$cfg.log; exit $rc; }
  python3 scripts/dispatch_order.py /tmp/r5_do20_$cfg | grep -E "wgemm|steps" | tee gpurun_out/r5_do20_$cfg.txt
done
echo ALLDONE
