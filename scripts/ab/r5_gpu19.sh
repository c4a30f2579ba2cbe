#!/bin/bash
# round-5 GPU session 19: per-dispatch kernel durations of cfg2 and rfstate with mep_wgemm_ws (which launch
# costs what) from a kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in cfg2 rfstate; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r5_do19_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/r5_do19_$cfg.log 2>&1; rc=$?
  echo "$cfg rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5_do19_$cfg.log; exit $rc; }
  python3 scripts/dispatch_order.py /tmp/r5_do19_$cfg | tee gpurun_out/r5_do19_$cfg.txt
done
echo ALLDONE
