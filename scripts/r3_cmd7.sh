#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/quick.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
for lib in variants/rff32/libmep_hip.so multimodal-emotion-processing_amd/libmep_hip.so; do
  MEP_LIB=$lib timeout -k 10 200 python3 bench.py --config cfg2 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/cfg2_ab.log 2>&1; rc=$?
  echo "== $lib cfg2 rc=$rc: $(tail -1 gpurun_out/cfg2_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], {k: v["ms_per_step"] for k, v in d["kernels"].items()})')"
  case $rc in 0) ;; *) exit $rc;; esac
done
NAMES="epi128 epione" KS=mep_block_epi_fwd,mep_block_epi_bwd CFGS="cfg3 cfg5" PARITY=1 bash scripts/r3_ab.sh || exit $?
echo "== default lib epilogues:"; timeout -k 10 120 python3 scripts/kbench.py --config cfg5 --kernel mep_block_epi_fwd,mep_block_epi_bwd --reps 20 2>&1 | grep us/launch
timeout -k 10 120 python3 scripts/kbench.py --config cfg3 --kernel mep_block_epi_fwd,mep_block_epi_bwd --reps 20 2>&1 | grep us/launch
bash scripts/bench_lines.sh
