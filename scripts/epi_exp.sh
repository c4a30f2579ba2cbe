#!/bin/bash
# A/B experiment: the forward epilogue built with MEP_EXP switches (csrc/block.hip), timed by
# scripts/kbench.py through the MEP_LIB override.  Development only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in ${EXPS:-0 1 2 4 8 3}; do
  make -s -C multimodal-emotion-processing_amd/csrc -j16 EXTRA="-DMEP_EXP=$e" BUILD=/tmp/mepexp$e OUT=/tmp/mepexp$e/lib.so > /dev/null 2>&1 || { echo "build $e failed"; exit 1; }
  echo "== MEP_EXP=$e"
  MEP_LIB=/tmp/mepexp$e/lib.so timeout -k 10 120 python3 scripts/kbench.py --kernel ${K:-mep_block_epi_fwd} --reps 50 || exit $?
done
