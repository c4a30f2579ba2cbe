#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "FATAL rc=$1"; exit $1;; esac; }
for v in e128 e128b1; do
  MEP_LIB=variants/$v/libmep_hip.so timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_$v.log 2>&1; rc=$?
  echo "== $v suite rc=$rc: $(tail -1 gpurun_out/pt_$v.log)"; grep FAILED gpurun_out/pt_$v.log; fatal $rc
done
NAMES="e128 e128b1" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS="cfg3 cfg5" bash scripts/r3_ab.sh
timeout -k 10 200 python3 scripts/diag/host_gap.py cfg3 > gpurun_out/hostgap.log 2>&1; fatal $?
timeout -k 10 200 python3 scripts/diag/host_gap.py cfg3 bf16 >> gpurun_out/hostgap.log 2>&1
grep -v amdgpu gpurun_out/hostgap.log
