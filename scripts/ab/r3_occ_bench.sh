#!/bin/bash
# bench lines, base vs variants/occ2, alternating, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do for cfg in cfg3 cfg2 cfg5; do for v in base occ2; do
  lib=""; [ $v != base ] && lib=variants/$v/libmep_hip.so
  MEP_LIB=$lib timeout -k 10 120 python3 bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ob.json 2>/dev/null || exit $?
  echo "$cfg $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ob.json)"
done; done; done
