#!/bin/bash
# A/B of prebuilt variants (scripts/build_variants.sh -> variants/<name>/libmep_hip.so) on the GPU box:
# per variant, kernel times of the attention launches at cfg3 and cfg5 (scripts/kbench.py), then
# (PARITY=1) the parity tests of the cmu / Ren-MME paths on that library.  Stops at a fatal status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "FATAL rc=$1"; exit $1;; esac; }
for name in ${NAMES:-$(ls variants)}; do
  lib=variants/$name/libmep_hip.so
  [ -f $lib ] || continue
  for cfg in ${CFGS:-cfg3 cfg5}; do
    for dt in ${DTYPES:-fp32}; do
      MEP_LIB=$lib timeout -k 10 120 python3 scripts/kbench.py --config $cfg --dtype $dt --kernel ${KS:-mep_attn_fwd,mep_attn_bwd} --reps ${REPS:-30} > gpurun_out/ab_$name.log 2>&1
      rc=$?; echo "== $name $cfg $dt: $(grep us/launch gpurun_out/ab_$name.log | tr -s ' ' | tr '\n' ';')"; fatal $rc
    done
  done
  if [ -n "$PARITY" ]; then
    MEP_LIB=$lib timeout -k 10 600 python3 -u -m pytest tests/test_gpu_cmu.py tests/test_gpu_ren.py -m gpu ${PX--x} -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_pt_$name.log 2>&1
    rc=$?; echo "== $name parity rc=$rc: $(tail -1 gpurun_out/ab_pt_$name.log)"; fatal $rc
  fi
done
exit 0
