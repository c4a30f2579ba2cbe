#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MEP_TGEMM=0 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_realformer.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rf_pt0.log 2>&1; rc=$?
echo "== realformer TGEMM=0 rc=$rc: $(tail -1 gpurun_out/rf_pt0.log)"; case $rc in 124|134|137|139) exit $rc;; esac
MEP_TGEMM_MIN_K=100000 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_realformer.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k cfg2 > gpurun_out/rf_pt1.log 2>&1; rc=$?
echo "== realformer MIN_K rc=$rc: $(tail -1 gpurun_out/rf_pt1.log)"; case $rc in 124|134|137|139) exit $rc;; esac
NAMES="base one" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS="cfg3" DTYPES="bf16 fp32" bash scripts/r3_ab.sh || exit $?
exit 0
