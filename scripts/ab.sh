#!/bin/bash
# A/B of compile-time kernel switches on the GPU box: VARIANTS="name=-DFLAG=1 -DX=2;name2=..." K=<launch>
# times K with scripts/kbench.py (MEP_LIB override) per variant.  Each variant's libmep_hip.so is
# variants/<name>/lib.so when present (built beforehand on the CPU host: scripts/ab_build.sh, it
# travels with the tree), else it is built into /tmp here.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  name=${v%%=*}; flags=${v#*=}
  lib=$PWD/variants/$name/lib.so
  if [ ! -f $lib ]; then
    lib=/tmp/ab_$name/lib.so
    make -s -C multimodal-emotion-processing_amd/csrc -j16 EXTRA="$flags" BUILD=/tmp/ab_$name OUT=$lib > /tmp/ab_$name.log 2>&1 || { echo "build $name failed"; tail -5 /tmp/ab_$name.log; exit 1; }
  fi
  for rep in 1 2; do
    echo "== $name ($flags) run $rep"
    MEP_LIB=$lib timeout -k 10 120 python3 scripts/kbench.py --kernel ${K:-mep_attn_bwd} --reps 100 $KARGS 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
