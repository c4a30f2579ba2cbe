#!/bin/bash
# Round-4 evidence passes, one rocprofv3 counter group per invocation, kernel
# trace only, never combined with other tracing:
#   1. FETCH_SIZE / WRITE_SIZE / TCC_EA0 request counters over scripts/micro/fetch_cal (known byte
#      counts per access width) -> the per-width correction (scripts/fetch_cal.py)
#   2. SQ instruction / cycle / MFMA / LDS-conflict groups over every kernel of the bench workloads
#      (cfg3, cfg3 bf16, cfg2, cfg5) -> per-kernel MFMA utilisation (scripts/r4_ctr_summary.py)
#   3. traffic: kernel trace + stats and the read / write byte counters per workload
#   STAGE=cal|sq|traffic|all CFGS="cfg3 cfg2 cfg5" bash scripts/r4_counters.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4ctr}
mkdir -p $OUT
STAGE=${STAGE:-all}
RD32="TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_sum"
pass() { local dir=$1; shift
  timeout -k 10 ${PT:-240} "$@" > $OUT/$dir.log 2>&1; local rc=$?
  echo "$dir rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/$dir.log; exit $rc;; esac; }
if [ $STAGE = cal ] || [ $STAGE = all ]; then
  test -x scripts/micro/fetch_cal || { echo "build scripts/micro/fetch_cal first"; exit 1; }
  pass cal_plain ./scripts/micro/fetch_cal
  pass cal_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/cal_fetch -o run --output-format csv -- ./scripts/micro/fetch_cal
  pass cal_write rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/cal_write -o run --output-format csv -- ./scripts/micro/fetch_cal
  pass cal_req rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $OUT/cal_req -o run --output-format csv -- ./scripts/micro/fetch_cal
  # bytes by request size: 32 B units of DRAM / GMI / IO read requests (a 64-B request counts 2,
  # a 128-B one 4)
  pass cal_req2 rocprofv3 --pmc $RD32 --kernel-trace -d $OUT/cal_req2 -o run --output-format csv -- ./scripts/micro/fetch_cal
fi
if [ $STAGE = traffic ] || [ $STAGE = all ]; then
  # per workload: kernel trace + stats, the 32-B read units and WRITE_SIZE (separate passes)
  for cfg in ${CFGS:-cfg3 cfg3_bf16 cfg2 cfg5 cfg5_bf16}; do
    case $cfg in
      cfg3) A="--config cfg3 --dtype fp32";; cfg3_bf16) A="--config cfg3 --dtype bf16";;
      cfg2) A="--config cfg2";; cfg5) A="--config cfg5 --dtype fp32";; cfg5_bf16) A="--config cfg5 --dtype bf16";;
      rfstate) A="--config rfstate";;
    esac
    # one precision per pass (kernel instances of the two paths share name prefixes), no HBM probe
    B="--steps ${PSTEPS:-30} --warmup 5 --no-cpu-baseline --no-bf16 --no-probe $A"
    pass ${cfg}_trace rocprofv3 --kernel-trace --stats -d $OUT/${cfg}_trace -o run --output-format csv -- python3 bench.py $B
    pass ${cfg}_rd rocprofv3 --pmc $RD32 --kernel-trace -d $OUT/${cfg}_rd -o run --output-format csv -- python3 bench.py $B
    pass ${cfg}_wr rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/${cfg}_wr -o run --output-format csv -- python3 bench.py $B
  done
fi
if [ $STAGE = sq ] || [ $STAGE = all ]; then
  G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
  G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32"
  G3="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"
  # keep only the counters this rocprofv3 lists (an unknown name fails the pass)
  timeout -k 10 120 rocprofv3 -L > $OUT/list.txt 2>&1 || true
  known() { local out=""; for c in $1; do grep -qw "$c" $OUT/list.txt && out="$out $c"; done; echo $out; }
  G4="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_READ_sum"   # L2 (round 6): hits / requests per kernel
  G1=$(known "$G1"); G2=$(known "$G2"); G3=$(known "$G3"); G4=$(known "$G4")
  echo "G1: $G1"; echo "G2: $G2"; echo "G3: $G3"; echo "G4: $G4"
  for cfg in ${CFGS:-cfg3 cfg3_bf16 cfg2 cfg5 cfg5_bf16}; do
    case $cfg in
      cfg3) A="--config cfg3 --dtype fp32";; cfg3_bf16) A="--config cfg3 --dtype bf16";;
      cfg2) A="--config cfg2";; cfg5) A="--config cfg5 --dtype fp32";; cfg5_bf16) A="--config cfg5 --dtype bf16";;
      rfstate) A="--config rfstate";;
    esac
    A="$A --no-bf16 --no-probe"
    i=0
    for grp in "$G1" "$G2" "$G3" ${SQ_L2:+"$G4"}; do
      i=$((i+1))
      pass ${cfg}_g$i rocprofv3 --pmc $grp --kernel-trace -d $OUT/${cfg}_g$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $A
    done
  done
fi
echo done
