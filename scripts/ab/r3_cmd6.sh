#!/bin/bash
# tiled GEMM tests first, then the full GPU suite, GEMM / epilogue A/B, bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tgemm.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_tgemm.log 2>&1
rc=$?; tail -15 gpurun_out/pt_tgemm.log; echo "tgemm tests rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
bash scripts/quick.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
for tg in 0 1; do echo "== MEP_TGEMM=$tg unify:"; for cfg in cfg3 cfg5; do MEP_TGEMM=$tg timeout -k 10 120 python3 scripts/kbench.py --config $cfg --kernel mep_unify --reps 20 2>&1 | grep us/launch; done; done
NAMES="epi128" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS=cfg5 PARITY=1 bash scripts/r3_ab.sh || exit $?
echo "== default lib epilogues:"; timeout -k 10 120 python3 scripts/kbench.py --config cfg5 --kernel mep_block_epi_fwd,mep_block_epi_bwd --reps 20 2>&1 | grep us/launch
bash scripts/bench_lines.sh
