#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_realformer.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rf_pt.log 2>&1; rc=$?
echo "== realformer rc=$rc: $(tail -1 gpurun_out/rf_pt.log)"; case $rc in 124|134|137|139) exit $rc;; esac
PX=" " NAMES="bwdonly all fwdwp3" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS="cfg3 cfg5" PARITY=1 bash scripts/r3_ab.sh || exit $?
for v in bwdonly all; do grep -E "FAILED|mismatch" gpurun_out/ab_pt_$v.log | head -20; done
exit 0
