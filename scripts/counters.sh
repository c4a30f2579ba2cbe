#!/bin/bash
# PMC passes on single kernels of the bench workload (scripts/kbench.py).  One counter group per
# rocprofv3 invocation, kernel trace only -- never combined with other tracing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctr
mkdir -p $OUT
K=${KERNELS:-"mep_attn_fwd mep_attn_bwd"}
timeout -k 10 120 rocprofv3 -L > $OUT/list.txt 2>&1 || true
CTR_GROUPS=${CTR_GROUPS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"}
i=0
IFS=';' read -ra GRPS <<< "$CTR_GROUPS"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  for k in $K; do
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $OUT/g${i}_$k -o run --output-format csv -- python3 scripts/kbench.py --kernel $k --reps 5 > $OUT/g${i}_$k.log 2>&1
    rc=$?; echo "group $i $k rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
timeout -k 10 200 python3 scripts/kbench.py --reps 50 > $OUT/kbench.log 2>&1; cat $OUT/kbench.log
