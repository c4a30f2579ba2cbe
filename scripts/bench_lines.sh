#!/bin/bash
# Bench lines of every BASELINE config on the GPU box -> gpurun_out/bench_<cfg>.json (one JSON line
# each; the fp32 lines and cfg2 carry the CPU baseline; the default dtype is the config's BASELINE one).  Stops at the first fatal exit status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$name.log 2>&1; local rc=$?
  grep -v amdgpu.ids gpurun_out/bench_$name.log | tail -1 > gpurun_out/bench_$name.json
  echo "== $name rc=$rc"; python3 -c "import json; d=json.load(open('gpurun_out/bench_$name.json')); print(d['value'], d['unit'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline_attention']['frac'], d.get('gpu_vs_cpu'))"
  case $rc in 0) ;; *) exit $rc;; esac; }
run cfg3 --steps 200 --warmup 20 --dtype fp32 --cpu-budget ${CPUB:-12}
run cfg3_bf16 --steps 200 --warmup 20 --dtype bf16 --cpu-budget ${CPUB:-12}
run cfg5 --config cfg5 --steps 50 --warmup 5 --dtype fp32 --cpu-budget ${CPUB:-12}
run cfg5_bf16 --config cfg5 --steps 50 --warmup 5 --dtype bf16 --cpu-budget ${CPUB:-12}
run cfg2 --config cfg2 --steps 200 --warmup 20 --cpu-budget ${CPUB:-12}
