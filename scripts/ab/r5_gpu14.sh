#!/bin/bash
# round-5 GPU session 14: the bf16 suite with its per-tensor error / budget ratios printed
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_cfg5_shape.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r5_t14.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "RAWBUDGET|worst tensors|bf16 |passed|failed" gpurun_out/r5_t14.log | head -60
echo ALLDONE
