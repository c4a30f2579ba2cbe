"""mep_wgrad_fused (csrc/gemm.hip k_wgrad<BF, true>): the weight gradients, their split sums, the
fusion-head parameter sums and the LayerNorm / residual-coefficient column sums in ONE launch,
against the two-launch form it replaces (mep_wgrad + mep_reduce_grads, trimodal.WGRAD_FOLD = 0):

- the flat gradient and the batch loss are bit-identical (the last arrival of a column group sums
  the group's slots in slot order, mep_wgrad_reduce's arithmetic), on the cfg3 shape (B = 64,
  T = 50, D = 96; fp32 and the bf16 path), a Ren-MME D = 128 shape with Tk > 64, the bucketed
  backward of the data-parallel engine, a realformer chain and a State_Transfer plan;
- every launch leaves the arrival tickets at zero, so graph replays and repeated backwards give
  the same gradients;
- the folded norm partials (one per column group and job workgroup) sum to the gradient's norm.
Reference: the weight-gradient half of loss.backward() and clip_grad_norm_'s norm
(cmu-mosei/run.py:367-368, others/realformer.py:340-341)."""
import pytest
import torch

from mep_amd import cmu_mosei, ren_mme, trimodal

pytestmark = pytest.mark.gpu


def _inputs(B, T, dims, NC, dev, seed=5):
    g = torch.Generator(device='cpu').manual_seed(seed)
    x = [torch.randn(B, 2, t, d, generator=g).to(dev) for t, d in zip(T, dims)]
    mk = [torch.ones(B, 2, t).to(dev) for t in T]
    mk[1][0, :, T[1] // 2:] = 0.0                      # a ragged row
    x[2][1] = 0.0                                      # an all-zero "no_name" row
    lab = (torch.rand(B, NC, generator=g) < 0.3).long().to(dev)
    return x, mk, lab


def _plan_grads(model, fold, B, T, dev, bf16=False, bucketed=False, reps=1):
    saved, trimodal.WGRAD_FOLD = trimodal.WGRAD_FOLD, fold
    try:
        r = model.mep_runner(dev)
        p = trimodal.TriModalPlan(r.spec, r.flat, B, T, dev, bf16=bf16)
        x, mk, lab = _inputs(B, T, r.spec.dims, r.spec.NC, dev)
        p.set_inputs(x[0], x[1], x[2], mk[0], mk[1], mk[2], lab)
        out = []
        for _ in range(reps):
            r.flat.grad.zero_()
            p.forward(grad=True)
            if bucketed:
                p.backward_bucketed(lambda: None)
            else:
                p.backward()
            torch.cuda.synchronize()
            out.append((r.flat.grad.clone(), p.loss.clone()))
        if fold:
            for arr in [p.d_wgrad] + ([p._buckets[0][1], p._buckets[1][1]] if bucketed else []):
                assert int(arr.tickets.abs().sum()) == 0, 'arrival tickets not left at zero'
    finally:
        trimodal.WGRAD_FOLD = saved
    return out


def _cmu(dev, D=96, H=6, T=(50, 50, 50), nl=1):
    return cmu_mosei.Concat_Trans(D, T[0], T[1], T[2], H, nl, 1).to(dev).eval()


@pytest.mark.parametrize('bf16', [False, True], ids=['fp32', 'bf16'])
def test_fused_wgrad_bit_exact_cfg3(bf16, cuda):
    torch.manual_seed(0)
    m = _cmu(cuda)
    (g0, l0), = _plan_grads(m, False, 64, (50, 50, 50), cuda, bf16=bf16)
    (g1, l1), (g2, l2) = _plan_grads(m, True, 64, (50, 50, 50), cuda, bf16=bf16, reps=2)
    assert torch.equal(l0, l1) and torch.equal(l1, l2)
    assert torch.equal(g0, g1), float((g0 - g1).abs().max())
    assert torch.equal(g1, g2), 'second backward differs: tickets not reset'


def test_fused_wgrad_bit_exact_ren_long(cuda):
    """Ren-MME (D = 128, MT = 4 tiles, unify K = 768 / 640 via mep_tgemm, LayerNorm column sums,
    9 classes) with Tk > 64"""
    torch.manual_seed(1)
    T = (8, 12, 80)
    m = ren_mme.Base_model(dim=128, l_len=T[0], v_len=T[1], a_len=T[2], n_heads=8, n_layers=1).to(cuda).eval()
    (g0, l0), = _plan_grads(m, False, 6, T, cuda)
    (g1, l1), = _plan_grads(m, True, 6, T, cuda)
    assert torch.equal(l0, l1)
    assert torch.equal(g0, g1), float((g0 - g1).abs().max())


def test_fused_wgrad_bit_exact_bucketed(cuda):
    """the data-parallel engine's two-bucket backward: both bucket launches fused"""
    torch.manual_seed(2)
    m = _cmu(cuda, D=32, H=2, T=(6, 9, 11), nl=2)
    (g0, _), = _plan_grads(m, False, 5, (6, 9, 11), cuda, bucketed=True)
    (g1, _), = _plan_grads(m, True, 5, (6, 9, 11), cuda, bucketed=True)
    (g2, _), = _plan_grads(m, True, 5, (6, 9, 11), cuda)
    assert torch.equal(g0, g1), float((g0 - g1).abs().max())
    assert torch.equal(g1, g2)


@pytest.mark.parametrize('family', ['chain', 'state'])
def test_fused_wgrad_bit_exact_realformer(family, cuda):
    from mep_amd import realformer as rf
    from mep_amd import rf_plan
    torch.manual_seed(3)
    B, P, T = 8, 3, 50
    if family == 'chain':
        mc = rf.Multi_class(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=T, v_len=T, a_len=T, n_heads=6,
                            n_layers=2, ffn=2).to(cuda)
        runner, PP = mc.mep_chain_runner(2, cuda), 1
        feats = (torch.randn(B, T, 300, device=cuda), torch.zeros(0, device=cuda), torch.zeros(0, device=cuda))
        masks = (torch.ones(B, T, device=cuda), torch.zeros(0, device=cuda), torch.zeros(0, device=cuda))
    else:
        st = rf.State_Transfer(300, 35, 74, 96, T, T, T, 6, 2, 2).to(cuda)
        runner, PP = st.mep_runner(cuda), P
        feats = tuple(torch.randn(B, P, T, d, device=cuda) for d in (300, 35, 74))
        masks = tuple((torch.rand(B, P, T, device=cuda) > 0.2).float() for _ in range(3))
    dout, grads = None, []
    for fold in (False, True, True):
        saved, trimodal.WGRAD_FOLD = trimodal.WGRAD_FOLD, fold
        try:
            plan = rf_plan.RealformerPlan(runner.spec, runner.flat, B, PP, cuda)
            plan.set_inputs(*feats, *masks)
            plan.forward(grad=True)
            if family == 'chain':
                if dout is None:
                    dout = torch.randn_like(plan.dout_chain)
                runner.flat.grad.zero_()
                plan.backward(ext_dout=dout)
            else:
                runner.flat.grad.zero_()
                plan.backward()
            torch.cuda.synchronize()
        finally:
            trimodal.WGRAD_FOLD = saved
        grads.append(runner.flat.grad.clone())
    assert torch.equal(grads[0], grads[1]), 'max |diff| %.3g' % (grads[0] - grads[1]).abs().max().item()
    assert torch.equal(grads[1], grads[2])


def test_fused_wgrad_norm_partials(cuda):
    """norm != 0: the launch writes one partial per column group and job workgroup, whose sum
    is ||grad||^2, and advances the optimizer step once"""
    from mep_amd import _lib
    torch.manual_seed(4)
    m = _cmu(cuda)
    r = m.mep_runner(cuda)
    p = trimodal.TriModalPlan(r.spec, r.flat, 64, (50, 50, 50), cuda)
    x, mk, lab = _inputs(64, (50, 50, 50), r.spec.dims, r.spec.NC, cuda)
    p.set_inputs(x[0], x[1], x[2], mk[0], mk[1], mk[2], lab)
    ws = torch.full((1024 + 4096,), float('nan'), device=cuda)
    step = torch.zeros(1, dtype=torch.int32, device=cuda)
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.01, 1.0, 0.0], device=cuda)
    p.norm_fold = (ws.data_ptr(), step.data_ptr(), hyper.data_ptr())
    saved, trimodal.WGRAD_FOLD = trimodal.WGRAD_FOLD, True
    try:
        n = p.reduce_grid()
        r.flat.grad.zero_()
        p.forward(grad=True)
        p.backward()
        torch.cuda.synchronize()
    finally:
        trimodal.WGRAD_FOLD = saved
    assert n == p.d_wgrad.n_cg + trimodal.fold_job_wg(
        trimodal.fold_jobs(p.d_colsum.n, p.t_colsum, p.head), p.t_wgrad, False)
    parts = ws[1024:1024 + n].double()
    assert bool(torch.isfinite(parts).all()), 'a norm partial was not written'
    assert bool(torch.isnan(ws[1024 + n:1024 + n + 16]).all()), 'a partial past n_ext was written'
    g = r.flat.grad[:r.flat.n_grad].double()
    want = float((g * g).sum())
    assert abs(float(parts.sum()) - want) <= 1e-5 * want
    assert int(step.item()) == 1
    assert _lib.lib().mep_abi_version() == _lib.ABI_VERSION
