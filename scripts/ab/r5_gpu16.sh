#!/bin/bash
# round-5 GPU session 16: compile-time knob A/B on cfg3 (fp32 + nested bf16): tgemm_n scheduling
# group (epilogues), waves per SIMD of the short attention backward (KV) and forward
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in main tg1 tg3 kv3 fw2 fw4; do
    if [ $v = main ]; then L=""; else L=variants/$v/libmep_hip.so; fi
    MEP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/r5_b16_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5_b16_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b16_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
k=d['kernels']; b=d['bf16']['kernels']
f=lambda x: ' '.join('%s %.1f'%(n.replace('mep_','').replace('block_','')[:9], x[n]['avg_launch_us']) for n in ('mep_attn_fwd','mep_attn_bwd','mep_block_epi_fwd','mep_block_epi_bwd'))
print('%-5s fp32 %.4f %s | bf16 %.4f %s'%(sys.argv[1], d['ms_per_step'], f(k), d['bf16']['ms_per_step'], f(b)))
PY
  done
done
echo ALLDONE
