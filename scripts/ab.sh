#!/bin/bash
# A/B of compile-time kernel switches on the GPU box: VARIANTS="name=-DFLAG=1 -DX=2;name2=..." K=<launch>
# builds each variant of libmep_hip.so into /tmp and times K with scripts/kbench.py (MEP_LIB override).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  name=${v%%=*}; flags=${v#*=}
  make -s -C multimodal-emotion-processing_amd/csrc -j16 EXTRA="$flags" BUILD=/tmp/ab_$name OUT=/tmp/ab_$name/lib.so > /tmp/ab_$name.log 2>&1 || { echo "build $name failed"; tail -5 /tmp/ab_$name.log; exit 1; }
  for rep in 1 2; do
    echo "== $name ($flags) run $rep"
    MEP_LIB=/tmp/ab_$name/lib.so timeout -k 10 120 python3 scripts/kbench.py --kernel ${K:-mep_attn_bwd} --reps 100 $KARGS 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
