"""bf16 path diagnostics on the GPU: per-tensor relative L2 error of the bf16 gradients against the
fp32 path's (whole tensors), for a fixture (scripts only; tests/test_gpu_bf16.py is the gate)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()
from tests.test_gpu_bf16 import _loss, _model_and_batch  # noqa: E402


def grads(name, bf16):
    dev = torch.device('cuda:0')
    meta, gold, model, args, labels = _model_and_batch(name, dev)
    model.mep_precision = 'bf16' if bf16 else 'fp32'
    model.train()
    logits = model(*args)
    _loss(meta, logits, labels).backward()
    return {k: p.grad.double().cpu() for k, p in model.named_parameters() if p.grad is not None}


for name in sys.argv[1:]:
    g32, g16 = grads(name, False), grads(name, True)
    errs = sorted(((float((g16[k] - g32[k]).norm() / g32[k].norm()), k) for k in g32), reverse=True)
    print(name, ' '.join('%s %.3f' % (k, e) for e, k in errs[:6]), flush=True)
    print('   median %.3f' % errs[len(errs) // 2][0])
