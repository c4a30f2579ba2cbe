"""GPU parity of the Ren-MME Base_model path (libmep_hip) against the reference golden vectors
(ren_small: D=32 H=2, full gradients; ren_full: D=128 H=8 T=(40,76,96), gradient norms/heads).

Tolerances as test_gpu_cmu.py: logits / loss rtol 1e-4; gradients rtol 1e-3 (floor 1e-5 x
max|grad|); post-AdamW parameters atol 2e-5 except where the reference gradient is at
rounding-noise level (gpu_util.check_post_params).  With DROP = 0 the duplicated rows make the
R-Drop KL and its gradient ~0 here; test_rdrop_head_vs_torch checks the fused KL on distinct
rows against a torch fp32 statement of Ren-MME/run.py:332-334.  The loss is multi_loss + the R-Drop KL of
Ren-MME/run.py:331-334 (the fixtures ran with DROP = 0, so the duplicated rows agree and the KL
is evaluated, not sampled).  Dropout itself (DROP > 0) uses a device hash, not torch's RNG, so it
is tested for its statistics and determinism instead of bit parity.
"""
import pytest
import torch

from tests.golden import fixtures
from tests.gpu_util import OUT_ATOL_FRAC, assert_close, check_post_params, ren_model

pytestmark = pytest.mark.gpu
REN = [n for n in fixtures.names('model') if fixtures.load(n)[0]['family'] == 'ren']


def _batch(meta, dev):
    inputs, labels = fixtures.batch(meta)
    return [t.to(dev) for t in inputs], labels.to(dev)


def _check_grads(model, meta, gold, coef):
    for k, p in model.named_parameters():
        if 'nograd/' + k in gold:
            assert p.grad is None, k
            continue
        g = p.grad * coef
        if meta['full']:
            assert_close(g, gold['grad/' + k], 1e-3, 1e-5, k)
        else:
            assert_close(g.reshape(-1)[:256], gold['gradhead/' + k], 1e-3, 1e-5, k)
            assert_close(torch.linalg.vector_norm(g.double()), gold['gradnorm/' + k], 1e-3, 0, k)


@pytest.mark.parametrize('name', REN)
def test_base_model_autograd(name, cuda):
    from mep_amd import ren_mme
    meta, gold = fixtures.load(name)
    model = ren_model(meta, cuda)
    model.train()
    args, labels = _batch(meta, cuda)
    logits = model(*args)
    assert_close(logits, gold['logits'], 1e-4, OUT_ATOL_FRAC, 'logits')
    loss = ren_mme.multi_loss(logits, labels) + ren_mme.rdrop_kl(logits)
    assert_close(loss.reshape(()), gold['loss'], 1e-4, 0, 'loss')
    loss.backward()
    _check_grads(model, meta, gold, float(gold['clipcoef']))


@pytest.mark.parametrize('graph', [False, True])
@pytest.mark.parametrize('name', REN)
def test_base_model_engine_step(name, graph, cuda):
    from mep_amd import ren_mme
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    meta, gold = fixtures.load(name)
    model = ren_model(meta, cuda)
    model.train()
    opt = FusedAdamW(model, lr=1e-3)
    eng = TrainEngine(model, opt, clip=1.0, rdrop=True, graph=graph)
    args, labels = _batch(meta, cuda)
    l, v, a, lm, vm, am = ren_mme._pack(args)
    losses = [float(eng.step(l, v, a, lm, vm, am, labels).item()) for _ in range(meta['steps'])]
    assert_close(losses[0], gold['loss'], 1e-4, 0, 'loss')
    assert_close(opt.gnorm.reshape(()), gold['gnorm'], 1e-4, 0, 'gnorm')
    check_post_params(model, meta, gold)
    model.eval()
    with torch.no_grad():
        logits2 = model(*args)
    assert_close(logits2, gold['logits2'], 1e-3, 1e-5, 'logits2')


def test_base_model_dropout(cuda):
    """DROP = 0.1 in train mode: duplicated rows get different masks (what R-Drop needs), the
    same seed state reproduces, eval mode is exactly the no-dropout network."""
    meta, gold = fixtures.load('ren_small')
    model = ren_model(meta, cuda, drop=0.1)
    args, labels = _batch(meta, cuda)
    model.eval()
    with torch.no_grad():
        ev = model(*args)
    assert_close(ev, gold['logits'], 1e-4, 1e-6, 'eval logits')
    model.train()
    with torch.no_grad():
        t1 = model(*args)
        t2 = model(*args)
    assert torch.isfinite(t1).all()
    assert (t1[0::2] - t1[1::2]).abs().max() > 1e-4, 'duplicate rows share a dropout mask'
    assert (t1 - t2).abs().max() > 1e-4, 'dropout seed does not advance between forwards'
    assert (t1 - ev).abs().max() > 1e-4


def _seed_tensor(v):
    import numpy as np
    return int(np.array([v], dtype=np.uint64).view(np.int64)[0])


@pytest.mark.parametrize('name', ['ren_drop', 'ren_drop_long'])
def test_base_model_dropout_pinned(name, cuda):
    """DROP = 0.1 pinned against the reference (tests/golden/ren_drop.npz): the reference's
    Base_model ran with each block's nn.Dropout applying the repo's counter-hash masks
    (oracle/dropout.py) of the fixture's seed, so logits, loss and every gradient must match the
    HIP path with the same seed -- mask placement (proj output and block output,
    Ren-MME/run.py:209,213), the 1/(1-p) scale and the gradient routing are all pinned."""
    from mep_amd import ren_mme
    meta, gold = fixtures.load(name)
    model = ren_model(meta, cuda, drop=meta['drop']['p'])
    model.train()
    args, labels = _batch(meta, cuda)
    l, v, a, lm, vm, am = ren_mme._pack(args)
    runner = model.mep_runner(cuda)
    plan = runner.stage(l, v, a, lm, vm, am, labels)
    plan.set_dropout(meta['drop']['p'])
    plan.seed.fill_(_seed_tensor(meta['drop']['seed']))
    plan.forward(grad=True, rdrop=True)
    plan.backward()
    torch.cuda.synchronize()
    assert_close(plan.logits, gold['logits'], 1e-4, OUT_ATOL_FRAC, 'logits')
    assert_close(plan.loss.reshape(()), gold['loss'], 1e-4, 0, 'loss')
    coef = float(gold['clipcoef'])
    for k, _ in model.named_parameters():
        if 'nograd/' + k in gold:
            continue
        assert_close(runner.flat.view(runner.flat.grad, k) * coef, gold['grad/' + k], 1e-3, 1e-5, k)


@pytest.mark.parametrize('graph', [False, True])
@pytest.mark.parametrize('name', ['ren_drop', 'ren_drop_long'])
def test_base_model_dropout_engine_step(name, graph, cuda):
    """The fused engine's training step at DROP = 0.1 (seed advanced once before the forward, as
    every training step does) against the reference step on the same masks: loss, clip norm and
    post-AdamW parameters; then the eval-mode forward (no dropout) of the updated model."""
    from mep_amd import ren_mme
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    meta, gold = fixtures.load(name)
    model = ren_model(meta, cuda, drop=meta['drop']['p'])
    model.train()
    opt = FusedAdamW(model, lr=1e-3)
    eng = TrainEngine(model, opt, clip=1.0, rdrop=True, graph=graph)
    args, labels = _batch(meta, cuda)
    l, v, a, lm, vm, am = ren_mme._pack(args)
    plan = model.mep_runner(cuda).plan_for(l, v, a)
    plan.seed.fill_(_seed_tensor(meta['drop']['seed0']))
    loss = float(eng.step(l, v, a, lm, vm, am, labels).item())
    assert_close(loss, gold['loss'], 1e-4, 0, 'loss')
    assert_close(opt.gnorm.reshape(()), gold['gnorm'], 1e-4, 0, 'gnorm')
    check_post_params(model, meta, gold)
    model.eval()
    with torch.no_grad():
        logits2 = model(*args)
    assert_close(logits2, gold['logits2'], 1e-3, 1e-5, 'logits2')


def test_dropout_mask_statistics(cuda):
    """The device masks' statistics at p = 0.1 over the whole ren_ref batch: keep rate 0.9 within
    5 sigma, every kept element scaled by exactly float32(1) / float32(0.9), masks change with
    the seed, and the two rows of an R-Drop pair get different masks."""
    import numpy as np
    meta, _ = fixtures.load('ren_ref')
    model = ren_model(meta, cuda, drop=0.1)
    model.train()
    from mep_amd import ren_mme
    args, labels = _batch(meta, cuda)
    l, v, a, lm, vm, am = ren_mme._pack(args)
    runner = model.mep_runner(cuda)
    plan = runner.stage(l, v, a, lm, vm, am, labels)
    plan.set_dropout(0.1)
    plan.seed.fill_(12345)
    plan.forward(grad=False)
    torch.cuda.synchronize()
    # site 1 of every block: out = drop(LN(z)) -> recover the mask as out / LN(z)
    blk = plan.blocks[0]
    z = blk['Z'].double()
    mean, rstd = blk['estat'][:, 0:1].double(), blk['estat'][:, 1:2].double()
    pre = runner.flat.view(runner.flat.buf, blk['pre'] + 'norm2.weight').double()
    bias = runner.flat.view(runner.flat.buf, blk['pre'] + 'norm2.bias').double()
    y = (z - mean) * rstd * pre + bias
    out = plan.Xcat[0][:, plan.toff[blk['qm']]:plan.toff[blk['qm']] + blk['Tq'], blk['col']:blk['col'] + plan.spec.D]
    out = out.reshape(-1, plan.spec.D).double()
    keep = (out != 0)
    big = keep & (y.abs() > 0.05)           # ratio well conditioned (fp32 LN output vs the fp64 restatement)
    ratio = (out[big] / y[big])
    assert float((ratio - float(np.float32(1) / np.float32(0.9))).abs().max()) < 2e-5
    n = keep.numel()
    rate = float(keep.double().mean())
    assert abs(rate - 0.9) < 5 * (0.09 / n) ** 0.5, rate
    rows = keep.reshape(plan.B, blk['Tq'], -1)
    assert bool((rows[0::2] != rows[1::2]).any()), 'pair rows share a mask'
    plan.seed.fill_(54321)
    plan.forward(grad=False)
    torch.cuda.synchronize()
    out2 = plan.Xcat[0][:, plan.toff[blk['qm']]:plan.toff[blk['qm']] + blk['Tq'], blk['col']:blk['col'] + plan.spec.D]
    assert bool(((out2.reshape(-1, plan.spec.D) != 0) != keep).any()), 'mask does not depend on the seed'


def test_unify_dimension_standalone(cuda):
    """Unify_Dimension.forward standalone (Ren-MME/run.py:167-168) vs a torch fp32 statement."""
    from mep_amd import ren_mme
    torch.manual_seed(0)
    u = ren_mme.Unify_Dimension(64).to(cuda)
    with torch.no_grad():
        u.norm1.weight.uniform_(0.5, 1.5)
        u.norm1.bias.uniform_(-0.2, 0.2)
    xs = [torch.randn(3, t, d, device=cuda, requires_grad=True)
          for t, d in ((7, ren_mme.L_DIM), (9, ren_mme.V_DIM), (70, ren_mme.A_DIM))]
    ys = u(*xs)
    ref_u = ren_mme.Unify_Dimension(64).to(cuda)
    ref_u.load_state_dict(u.state_dict())
    xr = [x.detach().clone().requires_grad_(True) for x in xs]
    n = ref_u.norm1
    refs = [torch.nn.functional.layer_norm(torch.nn.functional.linear(x, w), (64,), n.weight, n.bias)
            for x, w in zip(xr, (ref_u.linguistic.weight, ref_u.visual.weight, ref_u.acoustic.weight))]
    gs = [torch.randn_like(r) for r in refs]
    for y, r in zip(ys, refs):
        assert_close(y, r, 1e-4, 1e-5, 'unify out')
    sum((y * g).sum() for y, g in zip(ys, gs)).backward()
    sum((r * g).sum() for r, g in zip(refs, gs)).backward()
    for x, r in zip(xs, xr):
        assert_close(x.grad, r.grad, 1e-3, 1e-5, 'dx')
    for (k, p), (_, q) in zip(u.named_parameters(), ref_u.named_parameters()):
        assert_close(p.grad, q.grad, 1e-3, 1e-5, k)


def test_rdrop_head_vs_torch(cuda):
    """Fused circle loss + R-Drop KL (mep_head_fwd_bwd, rdrop=1) against the reference's torch
    statement (Ren-MME/run.py:331-334) on the same encoder, with the two rows of every pair made
    different so the KL and its gradient are far from 0."""
    from mep_amd import ren_mme
    meta, _ = fixtures.load('ren_small')
    model = ren_model(meta, cuda)
    model.train()
    args, labels = _batch(meta, cuda)
    g = torch.Generator(device='cpu').manual_seed(5)
    args = [t.clone() for t in args]
    for i in (0, 2, 4, 6, 8, 10):   # features of odd rows perturbed (masks untouched)
        args[i][1::2] += 0.5 * torch.randn(args[i][1::2].shape, generator=g).to(cuda) * (args[i + 1][1::2, :, None])
    logits = model(*args)
    m_loss = ren_mme.multi_loss(logits, labels)
    kl = ren_mme.rdrop_kl(logits)
    assert float(kl) > 1e-3
    (m_loss + kl).backward()
    ref_loss = float(m_loss + kl)
    ref_grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    runner = model.mep_runner(cuda)
    l, v, a, lm, vm, am = ren_mme._pack(args)
    plan = runner.stage(l, v, a, lm, vm, am, labels)
    plan.set_dropout(0.0)
    plan.forward(grad=True, rdrop=True)
    plan.backward()
    torch.cuda.synchronize()
    assert_close(plan.loss.reshape(()), ref_loss, 1e-5, 0, 'loss')
    for k, gr in ref_grads.items():
        assert_close(runner.flat.view(runner.flat.grad, k), gr, 1e-4, 1e-5, k)
