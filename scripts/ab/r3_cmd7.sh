#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/quick.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
cfg2() {  # cfg2 bench line with the given env / library -> ms per step and per-kernel times
  timeout -k 10 200 python3 bench.py --config cfg2 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/cfg2_ab.log 2>&1; rc=$?
  echo "== cfg2 $1 rc=$rc: $(tail -1 gpurun_out/cfg2_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], {k: v["ms_per_step"] for k, v in d["kernels"].items()})')"
  return $rc
}
MEP_LIB=variants/rff32/libmep_hip.so MEP_TGEMM_RES=0 cfg2 "rf f32, old gemm" || exit $?
MEP_TGEMM_RES=0 cfg2 "rf split, old gemm" || exit $?
cfg2 "rf split, resident tgemm" || exit $?
for tg in "MEP_TGEMM=0" "MEP_TGEMM_RES=0" "X=1"; do echo "== $tg unify:"; for cfg in cfg3 cfg5; do env $tg timeout -k 10 120 python3 scripts/kbench.py --config $cfg --kernel mep_unify --reps 20 2>&1 | grep us/launch; done; done
NAMES="epi128 epione" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS="cfg3 cfg5" PARITY=1 bash scripts/r3_ab.sh || exit $?
echo "== default lib epilogues:"; for cfg in cfg3 cfg5; do timeout -k 10 120 python3 scripts/kbench.py --config $cfg --kernel mep_block_epi_fwd,mep_block_epi_bwd --reps 20 2>&1 | grep us/launch; done
bash scripts/bench_lines.sh
