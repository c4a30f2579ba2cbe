#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in pv1 pv0; do for cfg in cfg3 cfg5; do MEP_LIB=variants/$v/libmep_hip.so timeout -k 10 120 python3 scripts/kbench.py --config $cfg --kernel mep_attn_fwd --reps 20 2>&1 | grep us/launch | sed "s/^/$v $cfg /"; done; done
for cfg in cfg3 cfg5; do timeout -k 10 120 python3 scripts/kbench.py --config $cfg --kernel mep_attn_fwd --reps 20 2>&1 | grep us/launch | sed "s/^/pv2 $cfg /"; done
PYTEST_X=" " bash scripts/quick.sh
