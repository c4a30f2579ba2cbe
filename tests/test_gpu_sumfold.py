"""The per-modality gradient sums folded into the short attention backward
(mep_attn_bwd_desc.sum, csrc/attn.hip fold_sums) against the separate mep_sum_rows launch: the unit
that completes a (b, h) slice adds the slice's sources in source order, so the training steps must
agree bit for bit (losses, gradient norms, parameters) -- including graph replays, where the slice
counters must have re-armed themselves.  Reference: the gradient of each unified modality feature is
the sum over every chain that reads it (cmu-mosei/run.py:297-313)."""
import pytest
import torch

from tests.golden import fixtures
from tests.gpu_util import cmu_model, cuda_batch

pytestmark = pytest.mark.gpu


def _steps(meta, batch, cuda, fold, monkeypatch, bf16=False):
    from mep_amd import trimodal
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    monkeypatch.setattr(trimodal, 'SUM_FOLD', fold)
    model = cmu_model(meta, cuda)
    model.train()
    opt = FusedAdamW(model, lr=1e-3)
    eng = TrainEngine(model, opt, clip=1.0, graph=True)
    losses = [eng.step(*batch).clone() for _ in range(4)]
    torch.cuda.synchronize()
    plans = list(model.mep_runner(cuda).plans.values())
    assert plans and all(p.sum_fold == fold for p in plans), [p.sum_fold for p in plans]
    return model, torch.cat(losses), opt.gnorm.clone(), plans[0]


def test_sum_fold_bit_equal_cmu_cfg3(cuda, monkeypatch):
    meta, _ = fixtures.load('cmu_cfg3')
    batch = cuda_batch(meta, cuda)
    m1, l1, g1, p1 = _steps(meta, batch, cuda, True, monkeypatch)
    assert int(p1.sum_count.abs().sum()) == 0, 'slice counters not re-armed'
    m0, l0, g0, p0 = _steps(meta, batch, cuda, False, monkeypatch)
    assert torch.equal(l1, l0), (l1, l0)
    assert torch.equal(g1, g0), (g1, g0)
    for k in p0.dU:
        assert torch.equal(p1.dU[k], p0.dU[k]), k
    for (k, a), (_, b) in zip(m1.named_parameters(), m0.named_parameters()):
        assert torch.equal(a, b), k
