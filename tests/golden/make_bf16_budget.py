"""Error budget of the bf16 path: how far torch.autocast(bfloat16) of the reference arithmetic lands
from the fp32 golden vectors, per fixture and per parameter gradient (test infrastructure).

The oracle (oracle/, the CPU restatement pinned to the reference's own classes by
tests/test_oracle.py) runs one training step of each fixture under
torch.autocast('cpu', dtype=torch.bfloat16) -- bf16 matmul / linear operands AND outputs, fp32
softmax / LayerNorm -- and the relative errors of its logits, loss, gradients and post-AdamW
parameters against the fixture's fp32 values are written to bf16_budget.json.
tests/test_gpu_bf16.py holds the HIP bf16 path to this budget: on the same inputs it must be at
least about as accurate as torch's own bf16 execution of the reference model.

    python tests/golden/make_bf16_budget.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tests import oracle_runner  # noqa: E402
from tests.golden import fixtures  # noqa: E402

CASES = ['cmu_small_l2', 'cmu_cfg3', 'ren_small', 'ren_ref', 'ren_cfg5']
LR = 1e-3


def budget(name):
    meta, gold = fixtures.load(name)
    with torch.autocast('cpu', dtype=torch.bfloat16):
        out = oracle_runner.run_model_case(meta, steps=1)
    want = torch.as_tensor(gold['logits']).double()
    rec = {'logits': float((out['logits'].double() - want).abs().max() / want.abs().max()),
           'loss': abs(float(out['loss']) - float(gold['loss'])) / abs(float(gold['loss']))}
    grads, gg, rr = {}, [], []
    for k, g in out['grads'].items():
        if g is None or 'nograd/' + k in gold:
            continue
        ref = torch.as_tensor(gold[('grad/' if meta['full'] else 'gradhead/') + k]).double().reshape(-1)
        got = g.double().reshape(-1)[:ref.numel()]
        grads[k] = float((got - ref).norm() / max(float(ref.norm()), 1e-30))
        gg.append(got)
        rr.append(ref)
    rec['grads'] = grads
    rec['grad_all'] = float((torch.cat(gg) - torch.cat(rr)).norm() / torch.cat(rr).norm())
    n_ok = n_all = 0
    if meta['steps'] == 1:
        for k, p in out['post'].items():
            ref = gold['post/' + k] if meta['full'] else gold['posthead/' + k]
            ref = torch.as_tensor(ref).double().reshape(-1)
            err = (p.double().reshape(-1)[:ref.numel()] - ref).abs()
            n_ok += int((err <= 0.25 * LR).sum())
            n_all += err.numel()
        rec['post_frac'] = n_ok / n_all
    return rec


def main():
    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count() or 1)
    res = {}
    for name in CASES:
        res[name] = budget(name)
        print(name, 'logits %.2e loss %.2e grad_all %.2e' % (res[name]['logits'], res[name]['loss'],
                                                              res[name]['grad_all']), flush=True)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'bf16_budget.json'), 'w') as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
