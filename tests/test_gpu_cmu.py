"""GPU parity of the cmu-mosei Concat_Trans path (libmep_hip) against the reference golden vectors.

Tolerances (north star: logits within 1e-4 fp32 relative): logits / loss rtol 1e-4; gradients
rtol 1e-3 with an absolute floor of 1e-5 x max|grad| (fp32 sums of 3200 tokens in a different
order than MKL); post-AdamW parameters atol 2e-5 (= 2 % of lr: Adam normalises tiny gradients
to ~lr-sized steps, amplifying rounding on near-zero grads).
"""
import pytest
import torch

from tests.golden import fixtures
from tests.gpu_util import (OUT_ATOL_FRAC, assert_close, assert_scores, check_post_params, close_or_spread, cmu_model,
                            cuda_batch)

pytestmark = pytest.mark.gpu
CMU = [n for n in fixtures.names('model') if fixtures.load(n)[0]['family'] == 'cmu']


@pytest.mark.parametrize('name', CMU)
def test_concat_trans_autograd(name, cuda):
    from mep_amd import cmu_mosei
    meta, gold = fixtures.load(name)
    model = cmu_model(meta, cuda)
    model.train()
    l, v, a, lm, vm, am, labels = cuda_batch(meta, cuda)
    logits = model(l, v, a, lm, vm, am)
    assert_close(logits, gold['logits'], 1e-4, OUT_ATOL_FRAC, 'logits')
    loss = cmu_mosei.multi_circle_loss(logits, labels).mean()
    assert_close(loss.reshape(()), gold['loss'], 1e-4, 0, 'loss')
    loss.backward()
    coef = float(gold['clipcoef'])
    for k, p in model.named_parameters():
        if 'nograd/' + k in gold:
            assert p.grad is None, k
            continue
        g = p.grad * coef  # fixture holds post-clip gradients
        if meta['full']:
            close_or_spread(g, gold, 'grad/' + k, 1e-3, 1e-5)
        else:
            assert_close(g.reshape(-1)[:256], gold['gradhead/' + k], 1e-3, 1e-5, k)
            assert_close(torch.linalg.vector_norm(g.double()), gold['gradnorm/' + k], 1e-3, 0, k)


@pytest.mark.parametrize('graph', [False, True])
@pytest.mark.parametrize('name', CMU)
def test_concat_trans_engine_step(name, graph, cuda):
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    meta, gold = fixtures.load(name)
    model = cmu_model(meta, cuda)
    model.train()
    opt = FusedAdamW(model, lr=1e-3)
    eng = TrainEngine(model, opt, clip=1.0, graph=graph)
    batch = cuda_batch(meta, cuda)
    losses = [float(eng.step(*batch).item()) for _ in range(meta['steps'])]
    assert_close(losses[0], gold['loss'], 1e-4, 0, 'loss')
    if meta['steps'] == 1:
        assert_close(opt.gnorm.reshape(()), gold['gnorm'], 1e-4, 0, 'gnorm')
    check_post_params(model, meta, gold)
    model.eval()
    with torch.no_grad():
        logits2 = model(*batch[:6])
    assert_close(logits2, gold['logits2'], 1e-3, 1e-5, 'logits2')


BLOCKS = [n for n in fixtures.names('block') if fixtures.load(n)[0]['family'] in ('cmu', 'ren')]


@pytest.mark.parametrize('name', BLOCKS)
def test_attention_block_standalone(name, cuda):
    """cmu-mosei / Ren-MME Attention_Block.forward called directly, against the reference block:
    [B, Tk] key masks, mask=None, [B, Tq, Tk] masks (the general attention kernels), residual
    scores including the F7 coefficients c = -1.5 / -1, and Ren-MME's block in training mode at
    DROP = 0.1 (the block's seed state set to the fixture's; masks of oracle/dropout.py)."""
    import numpy as np
    from mep_amd import cmu_mosei, ren_mme
    meta, gold = fixtures.load(name)
    c = meta['ctor']
    mod = cmu_mosei if meta['family'] == 'cmu' else ren_mme
    blk = mod.Attention_Block(c['dim'], c['n_heads'], c['ffn'])
    from tests.gpu_util import load_params
    load_params(blk, meta)
    blk = blk.to(cuda).train()
    drop = meta.get('drop')
    blk.drop.p = drop['p'] if drop else 0.0
    if drop:
        blk._mep_seed = torch.tensor([drop['seed0'], 0], dtype=torch.int64, device=cuda)
    q, kv, mask, s_prev, g_out = fixtures.block_inputs(meta)
    qt = torch.tensor(q, device=cuda, requires_grad=True)
    kvt = torch.tensor(kv, device=cuda, requires_grad=True)
    sp = torch.tensor(s_prev, device=cuda, requires_grad=True) if s_prev is not None else None
    y, s = blk(qt, kvt, kvt, None if mask is None else torch.tensor(mask, device=cuda), sp)
    # D = 128 epilogues run on 2-part weights (<= 2^-17 relative per product): on
    # the LayerNorm-scaled output that is up to ~2^-17 absolute on an entry, 2^-18 of a block
    # output's max (|y| ~ 5); the D <= 96 blocks are on six products and keep the 1e-6 bound
    atol_out = 2.0 ** -18 if c['dim'] >= 128 else OUT_ATOL_FRAC
    assert_close(y, gold['out'], 1e-4, atol_out, 'out')
    assert_scores(s, gold, meta, blk.c.detach().cpu().numpy(), s_prev, mask, q, kv)
    obj = (y * torch.tensor(g_out, device=cuda)).sum()
    if meta['g_scores']:
        obj = obj + (s * torch.tensor(gold['g_scores'], device=cuda)).sum()
    obj.backward()
    close_or_spread(qt.grad, gold, 'grad_q', 1e-3, 1e-5)
    close_or_spread(kvt.grad, gold, 'grad_kv', 1e-3, 1e-5)
    if sp is not None:
        close_or_spread(sp.grad, gold, 'grad_sprev', 1e-3, 1e-5)
    for k, p in blk.named_parameters():
        if 'nograd/' + k in gold:
            assert p.grad is None, k
        else:
            close_or_spread(p.grad, gold, 'grad/' + k, 1e-3, 1e-5)
    assert np.isfinite(y.detach().cpu().numpy()).all()
