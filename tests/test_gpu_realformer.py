"""GPU parity of the others/realformer.py path (libmep_hip) against the reference golden vectors:
the standalone RealFormer Attention_Block (K != V projections, residual scores, a/b ReZero
scalars, FFN), the BASELINE cfg2 text chain (Conv1d unify + positions + 2 blocks, at the small
and the full D=96/T=50 shape) and the whole State_Transfer step (P utterances through the shared
encoder, sigmoid/tanh gate recurrence, masked circle loss, clip, Adam).

Tolerances as test_gpu_cmu.py: outputs rtol 1e-4, gradients rtol 1e-3 (floor 1e-5 x max|grad|),
post-Adam parameters atol 2e-5 (gpu_util.check_post_params).

State_Transfer outputs are compared on the real utterances (utterance mask 1).  The padding
utterances (mask 0, features and key masks all zero) have every attention row fully masked: the
reference evaluates softmax(s - 1e8), and s - 1e8 rounds to the fp32 grid of spacing 8 around
-1e8, so those rows' weights are set by the last ulps of s (a summation-order artefact of the
projections).  Their outputs are masked out of the loss and never feed a real utterance (the
gate recurrence runs forward and padding is trailing), so loss, gradients and updates are
unaffected; for them only finiteness is checked.
"""
import contextlib

import pytest
import torch

from tests.golden import fixtures
from tests.gpu_util import (assert_close, assert_scores, check_grad_budget, check_post_budget, check_post_params,
                            close_or_spread, has_fp32_budget, load_params)

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def ffn_const(meta):
    """Attention_Block reads the module constant FFN at construction (realformer.py:163-168)."""
    from mep_amd import realformer as rf
    old = rf.FFN
    rf.FFN = meta['consts']['FFN']
    try:
        yield rf
    finally:
        rf.FFN = old


RF_BLOCKS = [n for n in fixtures.names('block') if fixtures.load(n)[0]['family'] == 'realformer']


@pytest.mark.parametrize('name', RF_BLOCKS)
def test_realformer_block_standalone(name, cuda):
    """block_rf, the F7 fixtures block_rf_f7_m15 / _m1 (c = -1.5 / -1: the masked slots carry the
    row's maximum / lose their -1e8; make_golden.py F7), and the other mask forms the reference
    accepts: mask=None (block_rf_nomask) and [B, Tq, Tk] (block_rf_mask3, the general kernels)"""
    meta, gold = fixtures.load(name)
    with ffn_const(meta) as rf:
        blk = rf.Attention_Block(meta['ctor']['dim'], meta['ctor']['n_heads'])
    load_params(blk, meta)
    blk = blk.to(cuda).train()
    q, kv, mask, s_prev, g_out = fixtures.block_inputs(meta)
    qt = torch.tensor(q, device=cuda, requires_grad=True)
    kvt = torch.tensor(kv, device=cuda, requires_grad=True)
    sp = torch.tensor(s_prev, device=cuda, requires_grad=True)
    y, s = blk(qt, kvt, kvt, None if mask is None else torch.tensor(mask, device=cuda), sp)
    close_or_spread(y, gold, 'out', 1e-4, 1e-6)
    wq, wk = (blk.w_qkv[i].weight.detach().double().cpu().numpy() for i in (0, 1))
    assert_scores(s, gold, meta, blk.c.detach().cpu().numpy(), s_prev, mask, q @ wq.T, kv @ wk.T)
    obj = (y * torch.tensor(g_out, device=cuda)).sum() + (s * torch.tensor(gold['g_scores'], device=cuda)).sum()
    obj.backward()
    close_or_spread(qt.grad, gold, 'grad_q', 1e-3, 1e-5)
    close_or_spread(kvt.grad, gold, 'grad_kv', 1e-3, 1e-5)
    close_or_spread(sp.grad, gold, 'grad_sprev', 1e-3, 1e-5)
    for k, p in blk.named_parameters():
        close_or_spread(p.grad, gold, 'grad/' + k, 1e-3, 1e-5)


@pytest.mark.parametrize('name', fixtures.names('chain'))
def test_text_chain(name, cuda):
    """BASELINE cfg2: realformer text encoder forward + backward of mean(out * G)."""
    meta, gold = fixtures.load(name)
    with ffn_const(meta) as rf:
        mc = rf.Multi_class(**meta['ctor'])
    load_params(mc, meta)
    mc = mc.to(cuda).train()
    x, lm, G = fixtures.chain_inputs(meta)
    out = rf.encode_chain(mc, torch.tensor(x, device=cuda), torch.tensor(lm, device=cuda), meta['n_layers'])
    assert_close(out, gold['out'], 1e-4, 1e-6, 'out')
    obj = (out * torch.tensor(G, device=cuda)).mean()
    assert_close(obj.reshape(()), gold['obj'], 1e-4, 1e-6, 'obj')
    obj.backward()
    for k, p in mc.named_parameters():
        if 'grad/' + k in gold:
            close_or_spread(p.grad, gold, 'grad/' + k, 1e-3, 1e-5)
        else:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k


def _check_out(out, want, um, rtol, atol_frac):
    """Every utterance slot, padded ones (um = 0) included: the reference returns outputs for all
    P slots (others/realformer.py:272-286) and the padded slots match too (3e-7 on rf_state_small)."""
    assert torch.isfinite(out).all()
    assert_close(out.detach().cpu(), torch.as_tensor(want), rtol, atol_frac, 'out')


def _state(meta, cuda):
    with ffn_const(meta) as rf:
        m = rf.State_Transfer(**meta['ctor'])
    load_params(m, meta)
    return m.to(cuda).train()


def _batch(meta, cuda):
    l, v, a, labels, lm, vm, am, um = [t.to(cuda) for t in fixtures.batch(meta)]
    return l, v, a, labels, lm, vm, am, um


STATE = ['rf_state_small', 'rf_state_ref']


def _check_state_grads(model, meta, gold, coef):
    """rf_state_small: every gradient at rtol 1e-3 (floor 1e-5 x max) against the reference.
    rf_state_ref (the reference's own configuration, others/realformer.py:23-38): its fp32
    gradients scatter around the exact values (near ties of the ReLU FFNs and max-pools over a
    6-step gate recurrence: the reference's own fp32 run lies up to 0.6% relative L2 from float64
    on some tensors), so each gradient is held against the reference in float64 to twice the
    fp32 budget the fixture measured over 12 reference and oracle executions
    (gpu_util.check_grad_budget), plus its norm within 1e-3 of the reference's."""
    budget = has_fp32_budget(gold)
    worst = 0.0
    for k, p in model.named_parameters():
        if 'nograd/' + k in gold:
            assert p.grad is None, k
            continue
        g = p.grad * coef
        if budget:
            worst = max(worst, check_grad_budget(g, gold, k, meta['full']))
            assert_close(torch.linalg.vector_norm(g.double()), gold['gradnorm/' + k], 1e-3, 0, k)
        elif meta['full']:
            assert_close(g, gold['grad/' + k], 1e-3, 1e-5, k)
        else:
            assert_close(g.reshape(-1)[:256], gold['gradhead/' + k], 1e-3, 1e-5, k)
            assert_close(torch.linalg.vector_norm(g.double()), gold['gradnorm/' + k], 1e-3, 0, k)
    if budget:
        print('worst gradient error / allowance: %.3f' % worst)


@pytest.mark.parametrize('name', STATE)
def test_state_transfer_autograd(name, cuda):
    from mep_amd import realformer as rf
    meta, gold = fixtures.load(name)
    model = _state(meta, cuda)
    l, v, a, labels, lm, vm, am, um = _batch(meta, cuda)
    out = model(l, v, a, lm, vm, am)
    _check_out(out, gold['logits'], um, 1e-4, 1e-6)
    loss = (rf.multi_circle_loss(out, labels) * um).mean()
    assert_close(loss.reshape(()), gold['loss'], 1e-4, 0, 'loss')
    loss.backward()
    _check_state_grads(model, meta, gold, float(gold['clipcoef']))


@pytest.mark.parametrize('graph', [False, True])
@pytest.mark.parametrize('name', STATE)
def test_state_transfer_engine_step(name, graph, cuda):
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdam
    meta, gold = fixtures.load(name)
    model = _state(meta, cuda)
    opt = FusedAdam(model, lr=1e-3)
    eng = TrainEngine(model, opt, clip=1.0, graph=graph)
    batch = _batch(meta, cuda)
    loss = float(eng.step(*batch).item())
    assert_close(loss, gold['loss'], 1e-4, 0, 'loss')
    assert_close(opt.gnorm.reshape(()), gold['gnorm'], 1e-4, 0, 'gnorm')
    if has_fp32_budget(gold):
        check_post_budget(model, meta, gold)
    else:
        check_post_params(model, meta, gold)
    l, v, a, labels, lm, vm, am, um = batch
    model.eval()
    with torch.no_grad():
        out2 = model(l, v, a, lm, vm, am)
    _check_out(out2, gold['logits2'], um, 1e-3, 1e-5)


def test_state_transfer_backward_twice_is_idempotent(cuda):
    """retain_graph: a second backward of one forward gives the same gradients (the rfw forward
    clears the attention dq rows once; a second backward clears them itself -- ADVICE r5)"""
    from mep_amd import realformer as rf
    meta, gold = fixtures.load('rf_state_small')
    model = _state(meta, cuda)
    l, v, a, labels, lm, vm, am, um = _batch(meta, cuda)
    out = model(l, v, a, lm, vm, am)
    loss = (rf.multi_circle_loss(out, labels) * um).mean()
    loss.backward(retain_graph=True)
    g1 = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    model.zero_grad(set_to_none=True)
    loss.backward()
    g2 = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    assert g1.keys() == g2.keys() and len(g1) > 10
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_state_transfer_wide_features_on_large_plans(cuda):
    """A State_Transfer plan big enough for mep_wgemm_ws (>= 8192 output tiles per launch) with a
    feature dim above its K <= 320 limit runs its unify on mep_wgemm: the logits of a
    B = 64 batch equal, row for row, those of a 2-row batch of the same sequences (rows are
    independent; the 2-row plan runs the small-launch kernels)."""
    from mep_amd import _lib
    from mep_amd import realformer as rf
    torch.manual_seed(3)
    T, P, B = 50, 6, 64
    old = rf.FFN
    rf.FFN = 2
    try:
        m = rf.State_Transfer(l_dim=400, v_dim=35, a_dim=74, dim=96, l_len=T, v_len=T, a_len=T, n_heads=6,
                              n_layers=2, ffn=2).to(cuda).eval()
    finally:
        rf.FFN = old
    g = torch.Generator(device='cpu').manual_seed(7)
    feats = [torch.randn(B, P, T, d, generator=g).to(cuda) for d in (400, 35, 74)]
    masks = [torch.ones(B, P, T, device=cuda) for _ in range(3)]
    with torch.no_grad():
        big = m(*feats, *masks)
        small = m(*[f[:2] for f in feats], *[k[:2] for k in masks])
    plan = m.mep_runner(cuda).plan(B, P)
    assert _lib.wgemm_tiles(plan.d_unify.items) >= _lib.WGEMM_WS_MIN
    assert plan.gemm_launcher(plan.d_unify) == 'mep_wgemm'
    assert torch.isfinite(big).all()
    assert_close(big[:2], small.cpu(), 1e-5, 1e-7, 'logits')
