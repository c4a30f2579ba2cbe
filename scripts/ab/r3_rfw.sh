#!/bin/bash
# realformer wave-kernel session: GPU suite (no -x), smoke, cfg2 bench on both kernel sets.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pt.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/pt.log | tail -n 40; echo "pytest rc=$rc"
fatal $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/smoke.log | tail -n 5; echo "smoke rc=$rc"
fatal $rc && exit $rc
for v in 1 0; do
  MEP_RFW=$v timeout -k 10 300 python bench.py --config cfg2 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_cfg2_rfw$v.log 2>&1
  rc=$?; echo "cfg2 rfw=$v rc=$rc"; grep -v amdgpu.ids gpurun_out/b_cfg2_rfw$v.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
  fatal $rc && exit $rc
done
exit 0
