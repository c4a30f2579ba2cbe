#!/bin/bash
# tests on the default library, then the D = 128 split epilogue A/B + parity, then bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/quick.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
NAMES="epi128" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS=cfg5 PARITY=1 bash scripts/r3_ab.sh || exit $?
echo "== default lib epilogues:"; MEP_LIB=multimodal-emotion-processing_amd/libmep_hip.so timeout -k 10 120 python3 scripts/kbench.py --config cfg5 --kernel mep_block_epi_fwd,mep_block_epi_bwd --reps 20 2>&1 | grep us/launch
bash scripts/bench_lines.sh
