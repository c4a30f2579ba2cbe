#!/bin/bash
# A/B of run-time plan switches on the GPU box: VARIANTS="name=ENV=1 ENV2=2;name2=..." -> bench.py
# (no CPU baseline) per variant, twice, one JSON line each; ARGS adds bench.py options.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  name=${v%%=*}; envs=${v#*=}
  for rep in 1 2; do
    echo "== $name ($envs) run $rep"
    env $envs timeout -k 10 180 python3 bench.py --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline $ARGS 2>&1 \
      | grep -v amdgpu.ids | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])" || exit $?
  done
done
