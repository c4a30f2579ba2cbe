#!/bin/bash
# round-5 GPU session 33: what folding the per-modality sums into the weight-gradient launch would
# cost (MEP_DEV_SUMFOLD_PROBE: the unify weight gradient as one item per source, no mep_sum_rows;
# timing only, wrong gradients) against the production step, cfg3 fp32 + bf16
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1; do
    MEP_DEV_SUMFOLD_PROBE=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/r5_b33_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5_b33_$v.log; exit 1; }
    python3 - $v <<'PY'
import json,sys
d=json.loads(open('gpurun_out/r5_b33_%s.log'%sys.argv[1]).read().strip().splitlines()[-1])
g=lambda x, n: x[n]['avg_launch_us'] if n in x else 0
for tag, x in (('fp32', d), ('bf16', d['bf16'])):
    k = x['kernels']
    print('probe=%s %s %.4f ms  wgrad %.1f  sum_rows %.1f  reduce %.1f' % (sys.argv[1], tag, x['ms_per_step'], g(k,'mep_wgrad'), g(k,'mep_sum_rows'), g(k,'mep_reduce_grads')))
PY
  done
done
echo ALLDONE
