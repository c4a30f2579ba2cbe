"""GPU check of the data-parallel step arithmetic: an N-rank step equals a 1-rank
step on the concatenated batch.  On one GPU the ranks are emulated: each share of the global
batch runs the fused forward + backward with the loss scaled to its part of the global mean
(plan.set_global_rows, as TrainEngine does under data parallelism), and the SUM of the shares'
flat gradients -- what the RCCL all-reduce computes -- must equal the full batch's gradient.
Shares are unequal (the ragged last batch) and, for Ren-MME, whole duplicate pairs (the R-Drop KL
batchmean divisor is the global pair count)."""
import pytest
import torch

from tests.golden import fixtures
from tests.gpu_util import assert_close, cmu_model, cuda_batch, ren_model

pytestmark = pytest.mark.gpu


def _grads(runner, batch, global_rows, drop=None, row0=0):
    """drop = (p, seed): the blocks' dropout at probability p with the seed state set to seed and
    the share's first global row row0 (engine.step_plan's set_row0)."""
    plan = runner.stage(*batch)
    plan.set_dropout(0.0 if drop is None else drop[0])
    if drop is not None:
        plan.seed.fill_(drop[1])
        plan.set_row0(row0)
    plan.set_global_rows(global_rows)
    plan.forward(grad=True, rdrop=runner.spec.variant == 'ren')
    plan.backward()
    torch.cuda.synchronize()
    return runner.flat.grad.clone(), float(plan.loss.item())


def _check(runner, full, shares, drop=None):
    g_full, l_full = _grads(runner, full, None, drop)
    n = full[-1].shape[0]                          # labels: one row per batch row
    g_sum, l_sum = torch.zeros_like(g_full), 0.0
    row0 = 0
    for s in shares:
        g, l = _grads(runner, s, n, drop, row0)
        row0 += s[-1].shape[0]
        g_sum += g
        l_sum += l
    n_grad = runner.flat.n_grad
    assert abs(l_sum - l_full) <= 1e-5 * abs(l_full)
    assert_close(g_sum[:n_grad], g_full[:n_grad], 1e-4, 1e-5, 'summed share gradients')


def test_dp_shares_sum_to_full_batch_cmu(cuda):
    meta, _ = fixtures.load('cmu_cfg1')            # B = 8, T = 50, D = 96
    model = cmu_model(meta, cuda)
    model.train()
    runner = model.mep_runner(cuda)
    full = cuda_batch(meta, cuda)
    cut = 5                                       # shares of 5 and 3 rows
    shares = [[t[:cut] for t in full], [t[cut:] for t in full]]
    _check(runner, full, shares)


def test_dp_shares_sum_to_full_batch_ren(cuda):
    from mep_amd import ren_mme
    meta, _ = fixtures.load('ren_small')           # 3 duplicate pairs = 6 rows
    model = ren_model(meta, cuda)
    model.train()
    runner = model.mep_runner(cuda)
    inputs, labels = fixtures.batch(meta)
    inputs = [t.clone() for t in inputs]
    g = torch.Generator().manual_seed(5)
    for i in (0, 2, 4, 6, 8, 10):   # the odd row of every duplicate pair perturbed (masks kept):
        inputs[i][1::2] += 0.5 * torch.randn(inputs[i][1::2].shape, generator=g) * inputs[i + 1][1::2, :, None]
    packed = list(ren_mme._pack([t.to(cuda) for t in inputs])) + [labels.to(cuda)]

    def rows(lo, hi):
        out = []
        for t in packed:
            if isinstance(t, (tuple, list)):
                out.append(type(t)(x[lo:hi] for x in t))
            else:
                out.append(t[lo:hi])
        return out
    full = rows(0, 6)                              # the R-Drop KL is far from 0 now
    _check(runner, full, [rows(0, 4), rows(4, 6)])
    # DROP = 0.1 (Ren-MME/run.py:36): with the shares' global row offsets every rank draws the
    # full batch's masks, so the SUM of the share gradients is still the full-batch gradient
    _check(runner, full, [rows(0, 4), rows(4, 6)], drop=(0.1, 987654321))
    _check(runner, full, [rows(0, 2), rows(2, 4), rows(4, 6)], drop=(0.1, 123456789))


def test_dp_dropout_masks_follow_global_rows(cuda):
    """A share's block outputs equal the full batch's rows row0 .. row0 + n (same seed, DROP = 0.1),
    and differ from the masks of local row indexing."""
    from mep_amd import ren_mme
    meta, _ = fixtures.load('ren_small')
    model = ren_model(meta, cuda)
    model.train()
    runner = model.mep_runner(cuda)
    inputs, labels = fixtures.batch(meta)
    packed = list(ren_mme._pack([t.to(cuda) for t in inputs])) + [labels.to(cuda)]

    def rows(lo, hi):
        return [type(t)(x[lo:hi] for x in t) if isinstance(t, (tuple, list)) else t[lo:hi] for t in packed]

    def xcat(batch, row0):
        plan = runner.stage(*batch)
        plan.set_dropout(0.1)
        plan.seed.fill_(424242)
        plan.set_row0(row0)
        plan.forward(grad=False)
        torch.cuda.synchronize()
        return [x.clone() for x in plan.Xcat]

    full = xcat(rows(0, 6), 0)
    share = xcat(rows(2, 6), 2)
    local = xcat(rows(2, 6), 0)
    for e in range(2):
        assert torch.equal(share[e], full[e][2:6]), 'share masks must be the full batch rows 2..5'
        assert not torch.equal(local[e], full[e][2:6]), 'row0 must change the masks'
