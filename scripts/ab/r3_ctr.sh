#!/bin/bash
# SQ counters of the cfg5 / cfg3 attention kernels (scripts/kbench.py; one counter group per rocprofv3
# --pmc pass, kernel trace only).  ENVS="name=VAR=val ..." selects library variants / env switches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctr
mkdir -p $OUT
CTR_GROUPS=${CTR_GROUPS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAIT_INST_LDS;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"}
IFS=';' read -ra GRPS <<< "$CTR_GROUPS"
for run in ${RUNS:-"wide:cfg5:mep_attn_bwd:MEP_ATTN_WIDE=1" "long:cfg5:mep_attn_bwd:MEP_ATTN_WIDE=0" "fwd:cfg5:mep_attn_fwd:X=1"}; do
  IFS=':' read -r tag cfg k env <<< "$run"
  i=0
  for grp in "${GRPS[@]}"; do
    i=$((i+1))
    ( export $env; timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/${tag}_g$i -o run --output-format csv -- python3 scripts/kbench.py --config $cfg --kernel $k --reps 3 > $OUT/${tag}_g$i.log 2>&1 )
    rc=$?; echo "$tag group $i rc=$rc"
    case $rc in 0) ;; *) tail -5 $OUT/${tag}_g$i.log; exit $rc;; esac
  done
done
exit 0
