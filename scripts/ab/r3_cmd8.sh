#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/quick.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
NAMES="both" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS="cfg3 cfg5" PARITY=1 bash scripts/r3_ab.sh || exit $?
for v in both; do MEP_LIB=variants/$v/libmep_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_dp.py tests/test_gpu_rccl.py tests/test_checkpoint.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_pt2_$v.log 2>&1; echo "== $v more parity rc=$?: $(tail -1 gpurun_out/ab_pt2_$v.log)"; done
for sq in 0 1; do echo "== MEP_FWD_SPLITQ=$sq:"; for cfg in cfg3 cfg5; do for dt in fp32 bf16; do MEP_FWD_SPLITQ=$sq timeout -k 10 120 python3 scripts/kbench.py --config $cfg --dtype $dt --kernel mep_attn_fwd --reps 20 2>&1 | grep us/launch | sed "s/^/$cfg $dt /"; done; done; done
