#!/bin/bash
# A/B of k_wgrad variants built with MEP_EXP switches into exp_build/ (development only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-base 256 512}; do
  echo "== $v"
  if [ "$v" = base ]; then L=""; else L=$PWD/exp_build/lib$v.so; fi
  MEP_LIB=$L timeout -k 10 120 python3 scripts/wgrad_exp.py ${WGARGS} 2>&1 | grep -v amdgpu.ids || exit $?
done
