"""Standalone encoder entries on the GPU: cmu-mosei / Ren-MME Multi_ATTN.forward and realformer
Multi_class.forward (reference code calls them directly: cmu-mosei/run.py:330-331,
Ren-MME/run.py:283-284, others/realformer.py:276).  Each runs the HIP unify and block kernels;
its logits and every parameter / input gradient are checked against the CPU oracle, which is
itself pinned to the reference's golden vectors (tests/test_oracle.py).  Tolerances as the model
tests: outputs rtol 1e-4, gradients rtol 1e-3 with a floor of 1e-4 x max (the backward's products
use 2-way bf16 splits, <= 2^-16 relative each -- csrc/attn.hip)."""
import pytest
import torch

from tests.golden import fixtures
from tests.gpu_util import OUT_ATOL_FRAC, assert_close, cmu_model, ren_model

pytestmark = pytest.mark.gpu


def _check(enc, pre, oracle_fn, inputs_cpu, meta, cuda):
    P = fixtures.params(meta)
    xs = [x.clone().requires_grad_(i < 3) for i, x in enumerate(inputs_cpu)]
    out_ref = oracle_fn(P, pre, *xs)
    G = torch.randn(out_ref.shape, generator=torch.Generator().manual_seed(3))
    (out_ref * G).sum().backward()
    xg = [x.to(cuda).detach().clone().requires_grad_(i < 3) for i, x in enumerate(inputs_cpu)]
    out = enc(*xg)
    assert_close(out, out_ref.detach(), 1e-4, OUT_ATOL_FRAC, 'output')
    (out * G.to(cuda)).sum().backward()
    for k, p in enc.named_parameters():
        ref = P[pre + k].grad
        if ref is None or float(ref.abs().max()) == 0.0:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k
            continue
        assert_close(p.grad, ref, 1e-3, 1e-4, k)
    for i in range(3):
        keep = inputs_cpu[3 + i].to(torch.bool)                     # [B, T], 1 = real step
        got, want = xg[i].grad.cpu(), xs[i].grad
        assert_close(got[keep], want[keep], 1e-3, 1e-4, 'input %d (real steps)' % i)
        # Padded steps carry identical features, so their block outputs tie (bit-exactly on the
        # GPU, to rounding on the CPU) and max-pool routes a row's gradient to one of them: the
        # reference's own choice among near-ties is BLAS-rounding noise.  What is invariant is
        # the sum over a row's padded steps.
        pad = (~keep).unsqueeze(-1).to(got.dtype)
        assert_close((got * pad).sum(1), (want * pad).sum(1), 1e-3, 1e-4, 'input %d (padded sum)' % i)


def test_multi_attn_forward_cmu(cuda):
    from oracle import cmu_mosei as ocmu
    meta, _ = fixtures.load('cmu_small_l2')        # two layers: residual scores between blocks
    model = cmu_model(meta, cuda)
    l, v, a, lm, vm, am, _ = fixtures.batch(meta)
    inputs = [l[:, 1], v[:, 1], a[:, 1], lm[:, 1], vm[:, 1], am[:, 1]]   # the current utterance
    H, nl = meta['ctor']['n_heads'], meta['ctor']['n_layers']
    _check(model.stimulation, 'stimulation.',
           lambda P, pre, *x: ocmu.multi_attn(P, pre, *x, n_heads=H, n_layers=nl), inputs, meta, cuda)


def test_multi_attn_forward_ren(cuda):
    from oracle import cmu_mosei as ocmu
    meta, _ = fixtures.load('ren_small')
    model = ren_model(meta, cuda)                  # DROP = 0 (the fixture's setting)
    model.train()
    inputs, _ = fixtures.batch(meta)
    ptf, ptm, _, _, pvf, pvm, _, _, paf, pam, _, _ = inputs
    H, nl = meta['ctor']['n_heads'], meta['ctor']['n_layers']
    _check(model.intensity, 'intensity.',
           lambda P, pre, *x: ocmu.multi_attn(P, pre, *x, n_heads=H, n_layers=nl, norm='norm2', unify_norm='norm1'),
           [ptf, pvf, paf, ptm, pvm, pam], meta, cuda)


def test_multi_class_forward_realformer(cuda):
    from oracle import realformer as orf
    from tests.test_gpu_realformer import _state
    meta, _ = fixtures.load('rf_state_small')
    model = _state(meta, cuda)
    l, v, a, _, lm, vm, am, _ = fixtures.batch(meta)
    inputs = [l[:, 0], v[:, 0], a[:, 0], lm[:, 0], vm[:, 0], am[:, 0]]    # the first utterance
    H, nl = meta['ctor']['n_heads'], meta['ctor']['n_layers']
    _check(model.feature, 'feature.',
           lambda P, pre, *x: orf.multi_class(P, pre, *x, n_heads=H, n_layers=nl), inputs, meta, cuda)
