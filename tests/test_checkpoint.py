"""Checkpoint compatibility and optimizer-state resume.

Model checkpoints are the reference's own state_dict (same keys, shapes and order;
cmu-mosei/run.py:415,447); optimizer state is torch.optim.AdamW's state_dict layout.  A resumed
run (save after k steps, load into fresh objects, continue) must equal the uninterrupted run bit
for bit: every kernel of the step is deterministic -- including the attention backward at
Tk > 64 (ren_ref: audio Tk = 275, five key chunks), whose dQ is summed over key chunks in a fixed
order (csrc/attn.hip k_attn_bwd_long)."""
import io

import pytest
import torch

from tests.golden import fixtures
from tests.gpu_util import cmu_model, cuda_batch, ren_model

pytestmark = pytest.mark.gpu


def _engine(meta, cuda):
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    ren = meta['family'] == 'ren'
    model = ren_model(meta, cuda) if ren else cmu_model(meta, cuda)
    model.train()
    opt = FusedAdamW(model, lr=1e-3)
    return model, opt, TrainEngine(model, opt, clip=1.0, rdrop=ren, graph=True)


def _batch(meta, cuda):
    if meta['family'] != 'ren':
        return cuda_batch(meta, cuda)
    from mep_amd import ren_mme
    inputs, labels = fixtures.batch(meta)
    return list(ren_mme._pack([t.to(cuda) for t in inputs])) + [labels.to(cuda)]


@pytest.mark.parametrize('name', ['cmu_small', 'ren_ref'])
def test_resume_is_bit_exact(name, cuda):
    meta, _ = fixtures.load(name)
    batch = _batch(meta, cuda)
    model, opt, eng = _engine(meta, cuda)
    for _ in range(3):
        eng.step(*batch)
    want = {k: v.detach().clone() for k, v in model.state_dict().items()}

    m2, o2, e2 = _engine(meta, cuda)
    for _ in range(2):
        e2.step(*batch)
    buf = io.BytesIO()
    torch.save({'model': m2.state_dict(), 'optim': o2.state_dict()}, buf)
    buf.seek(0)
    ck = torch.load(buf, weights_only=True)
    assert list(ck['model']) == list(m2.state_dict())              # reference key order
    m3, o3, e3 = _engine(meta, cuda)
    m3.load_state_dict(ck['model'])
    o3.load_state_dict(ck['optim'])
    e3.step(*batch)
    for k, v in m3.state_dict().items():
        assert torch.equal(v, want[k]), k


def test_long_attention_backward_is_deterministic(cuda):
    """Two backward passes of the same Ren-MME step at Tk = 275 give bitwise equal gradients."""
    meta, _ = fixtures.load('ren_ref')
    batch = _batch(meta, cuda)
    model, opt, eng = _engine(meta, cuda)
    runner = model.mep_runner(cuda)
    plan = runner.stage(*batch)
    plan.set_dropout(0.0)
    grads = []
    for _ in range(2):
        plan.forward(grad=True, rdrop=True)
        plan.backward()
        torch.cuda.synchronize()
        grads.append(runner.flat.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_optimizer_state_is_torch_layout(cuda):
    meta, _ = fixtures.load('cmu_small')
    batch = cuda_batch(meta, cuda)
    model, opt, eng = _engine(meta, cuda)
    eng.step(*batch)
    eng.step(*batch)
    sd = opt.state_dict()
    params = list(model.parameters())
    assert sd['param_groups'][0]['params'] == list(range(len(params)))
    for i, p in enumerate(params):
        if i in sd['state']:
            s = sd['state'][i]
            assert float(s['step']) == 2.0
            assert s['exp_avg'].shape == p.shape and s['exp_avg_sq'].shape == p.shape
            assert bool((s['exp_avg_sq'] >= 0).all())
    # every parameter that gets a gradient has state; the first-layer residual coefficients c
    # (scores=None, cmu-mosei/run.py:243-246) never do and, as in torch, carry none
    names = [n for n, _ in model.named_parameters()]
    assert sorted(sd['state']) == [i for i, n in enumerate(names) if opt._flat.has_grad[n]]
    assert all(n.endswith('.c') for i, n in enumerate(names) if i not in sd['state'])
    # the same dict drives torch's own AdamW over CPU copies of the parameters
    cpu = [p.detach().cpu().clone().requires_grad_() for p in params]
    ref = torch.optim.AdamW(cpu, lr=1e-3)
    ref.load_state_dict(sd)
    assert float(ref.state[cpu[next(iter(sd['state']))]]['step']) == 2.0
    # and a torch AdamW state_dict loads back
    o2 = _engine(meta, cuda)[1]
    o2.load_state_dict(ref.state_dict())
    assert int(o2.step_t.item()) == 2
