#!/bin/bash
# round-5 GPU session 27: what the epilogue kernels' per-workgroup weight staging costs -- cfg3
# (fp32 + bf16) with a timing-only build that skips it (MEP_EPI_NOSTAGE: wrong results)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in main nostage; do
    if [ $v = main ]; then L=""; else L=variants/$v/libmep_hip.so; fi
    MEP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/r5_b27_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5_b27_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b27_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
k=d['kernels']; b=d['bf16']['kernels']
f=lambda x: ' '.join('%s %.1f'%(n.replace('mep_','').replace('block_','')[:9], x[n]['avg_launch_us']) for n in ('mep_block_epi_fwd','mep_block_epi_bwd'))
print('%-8s fp32 %.4f %s | bf16 %.4f %s'%(sys.argv[1], d['ms_per_step'], f(k), d['bf16']['ms_per_step'], f(b)))
PY
  done
done
echo ALLDONE
