"""The pool backward folded into the epilogue backward (trimodal.POOL_FOLD, csrc/block.hip
Upstream) against the separate mep_pool_bwd launch into dXcat: the same step on the same weights
and batch gives bit-identical block gradients and flat parameter gradients (the fold forms
exactly k_pool_bwd's dx: dmean / T, + dmax at the argmax step; cmu-mosei/run.py:314-318)."""
import pytest
import torch

from mep_amd import cmu_mosei, ren_mme, trimodal

pytestmark = pytest.mark.gpu


def _step(model, fold, B, T, dims, dev, NC):
    saved, trimodal.POOL_FOLD = trimodal.POOL_FOLD, fold
    try:
        r = model.mep_runner(dev)
        p = trimodal.TriModalPlan(r.spec, r.flat, B, T, dev)
    finally:
        trimodal.POOL_FOLD = saved
    assert p.pool_fold == fold
    g = torch.Generator(device='cpu').manual_seed(5)
    x = [torch.randn(B, 2, t, d, generator=g).to(dev) for t, d in zip(T, dims)]
    mk = [torch.ones(B, 2, t).to(dev) for t in T]
    mk[1][0, :, T[1] // 2:] = 0.0                      # a ragged row
    x[2][1] = 0.0                                      # an all-zero "no_name" row (max-pool ties)
    lab = (torch.rand(B, NC, generator=g) < 0.3).long().to(dev)
    p.set_inputs(x[0], x[1], x[2], mk[0], mk[1], mk[2], lab)
    r.flat.grad.zero_()
    p.forward(grad=True)
    p.backward()
    torch.cuda.synchronize()
    return r.flat.grad.clone(), [b['dZ'].clone() for b in p.blocks]


@pytest.mark.parametrize('family,nl', [('cmu', 1), ('cmu', 2), ('ren', 1)])
def test_pool_fold_is_bit_exact(family, nl, cuda):
    torch.manual_seed(0)
    T = (6, 9, 11)
    if family == 'cmu':
        m = cmu_mosei.Concat_Trans(32, T[0], T[1], T[2], 2, nl, 1)
    else:
        m = ren_mme.Base_model(dim=32, l_len=T[0], v_len=T[1], a_len=T[2], n_heads=2, n_layers=nl)
    m = m.to(cuda).eval()
    spec = m.mep_runner(cuda).spec
    dims, NC = spec.dims, spec.NC
    g0, z0 = _step(m, False, 4, T, dims, cuda, NC)
    g1, z1 = _step(m, True, 4, T, dims, cuda, NC)
    for i, (a, b) in enumerate(zip(z0, z1)):
        assert torch.equal(a, b), (i, float((a - b).abs().max()))
    assert torch.equal(g0, g1), float((g0 - g1).abs().max())
