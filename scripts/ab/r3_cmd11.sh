#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/quick.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
for v in pv1 pv0; do for cfg in cfg3 cfg5; do MEP_LIB=variants/$v/libmep_hip.so timeout -k 10 120 python3 scripts/kbench.py --config $cfg --kernel mep_attn_fwd --reps 20 2>&1 | grep us/launch | sed "s/^/$v $cfg /"; done; done
for cfg in cfg3 cfg5; do timeout -k 10 120 python3 scripts/kbench.py --config $cfg --kernel mep_attn_fwd --reps 20 2>&1 | grep us/launch | sed "s/^/pv2 $cfg /"; done
NAMES="one128" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS="cfg5" DTYPES="bf16" bash scripts/r3_ab.sh || exit $?
timeout -k 10 120 python3 scripts/kbench.py --config cfg5 --dtype bf16 --kernel mep_block_epi_fwd,mep_block_epi_bwd --reps 20 2>&1 | grep us/launch | sed "s/^/base cfg5 bf16 /"
MEP_LIB=variants/one128/libmep_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bf16.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_one128.log 2>&1; echo "== one128 bf16 rc=$?: $(tail -1 gpurun_out/pt_one128.log)"
exit 0
