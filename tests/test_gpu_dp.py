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


def _grads(runner, batch, global_rows):
    plan = runner.stage(*batch)
    plan.set_dropout(0.0)
    plan.set_global_rows(global_rows)
    plan.forward(grad=True, rdrop=runner.spec.variant == 'ren')
    plan.backward()
    torch.cuda.synchronize()
    return runner.flat.grad.clone(), float(plan.loss.item())


def _check(runner, full, shares):
    g_full, l_full = _grads(runner, full, None)
    n = full[-1].shape[0]                          # labels: one row per batch row
    g_sum, l_sum = torch.zeros_like(g_full), 0.0
    for s in shares:
        g, l = _grads(runner, s, n)
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
