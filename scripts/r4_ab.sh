#!/bin/bash
# Same-box A/B of bench lines: VARIANTS="name=ENV=1 ENV2=2;..." ARGS="--config cfg5" REPS=2
# -> gpurun_out/r4ab_<tag>.jsonl, one full bench JSON line per run (per-kernel times included)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-ab}
OUT=gpurun_out/r4ab_$TAG.jsonl
: > $OUT
IFS=';' read -ra VS <<< "$VARIANTS"
for rep in $(seq ${REPS:-2}); do
  for v in "${VS[@]}"; do
    name=${v%%=*}; envs=${v#*=}
    env $envs timeout -k 10 ${BT:-180} python3 bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline $ARGS > gpurun_out/r4ab_last.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 gpurun_out/r4ab_last.log; exit $rc; fi
    tail -1 gpurun_out/r4ab_last.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['ab']='$name'; print(json.dumps(d))" >> $OUT
    python3 -c "
import json; d=[json.loads(l) for l in open('$OUT')][-1]
k=d['kernels']; top=sorted(k.items(), key=lambda kv:-kv[1]['ms_per_step'])[:6]
print('$name', d['value'], d['ms_per_step'], ' '.join('%s=%.1fus' % (n.replace('mep_',''), 1e3*v['ms_per_step']/max(1,v['launches_per_step'])) for n,v in top))"
  done
done
