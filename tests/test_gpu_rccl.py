"""The data-parallel exchange on hardware: a world-1 ``nccl`` (= RCCL) process group
drives TrainEngine with the flat-gradient all-reduce CAPTURED in the step's hipGraph, between the
backward and the optimizer.  A SUM over one rank is the identity, so every step must equal the
no-data-parallel engine's bit for bit -- what this pins is that the RCCL call runs inside the
replayed graph, on the right buffer, in the right place of the step (before clip + AdamW).
Reference step: cmu-mosei/run.py:364-369 (backward, clip_grad_norm_, AdamW.step)."""
import socket

import pytest
import torch
import torch.distributed as dist

from tests.golden import fixtures
from tests.gpu_util import cmu_model, cuda_batch, ren_model

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture
def nccl_world1(cuda):
    if dist.is_initialized():
        pytest.skip('a process group already exists')
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % _free_port(), rank=0, world_size=1,
                            device_id=cuda)
    try:
        yield
    finally:
        dist.destroy_process_group()


def _run(model_fn, batch, steps, collective, rdrop=False, seed=None, fold_norm=False):
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    model = model_fn()
    model.train()
    opt = FusedAdamW(model, lr=1e-3)
    # the collective engine keeps the optimizer's own norm pass (the norm follows the SUM): the
    # engine it is compared with bit for bit does too
    eng = TrainEngine(model, opt, clip=1.0, rdrop=rdrop, graph=True, collective=collective, fold_norm=fold_norm)
    if seed is not None:
        model.mep_runner(batch[0][0].device if isinstance(batch[0], (tuple, list)) else batch[0].device) \
            .seed_state[0].fill_(seed)
    losses = [eng.step(*batch).clone() for _ in range(steps)]
    torch.cuda.synchronize()
    return eng, model, torch.cat(losses), opt.gnorm.clone()


def test_rccl_allreduce_captured_cmu_cfg3(nccl_world1, cuda):
    """BASELINE cfg3 shape (B = 64, T = 50): one eager step, then graph replays with the captured
    RCCL all-reduce; equal to the engine without the collective."""
    meta, _ = fixtures.load('cmu_cfg3')
    batch = cuda_batch(meta, cuda)
    e1, m1, l1, g1 = _run(lambda: cmu_model(meta, cuda), batch, 4, collective=True)
    assert e1.collective and e1.capture_allreduce, 'the RCCL all-reduce was not captured in the graph'
    assert all(b is None for (_, b) in e1._graphs.values()), 'expected one graph per step'
    e0, m0, l0, g0 = _run(lambda: cmu_model(meta, cuda), batch, 4, collective=False)
    assert not e0.collective
    assert torch.equal(l1, l0), (l1, l0)
    assert torch.equal(g1, g0)
    for (k, p1), (_, p0) in zip(m1.named_parameters(), m0.named_parameters()):
        assert torch.equal(p1, p0), k


def test_rccl_allreduce_captured_ren_dropout(nccl_world1, cuda):
    """Ren-MME at DROP = 0.1 (the seed advances inside the captured graph) through the captured
    all-reduce, with the R-Drop head."""
    from mep_amd import ren_mme
    meta, _ = fixtures.load('ren_drop_long')
    inputs, labels = fixtures.batch(meta)
    batch = list(ren_mme._pack([t.to(cuda) for t in inputs])) + [labels.to(cuda)]
    p = meta['drop']['p']
    e1, m1, l1, g1 = _run(lambda: ren_model(meta, cuda, drop=p), batch, 3, True, rdrop=True, seed=77)
    assert e1.capture_allreduce
    e0, m0, l0, g0 = _run(lambda: ren_model(meta, cuda, drop=p), batch, 3, False, rdrop=True, seed=77)
    assert torch.equal(l1, l0) and torch.equal(g1, g0)
    for (k, p1), (_, p0) in zip(m1.named_parameters(), m0.named_parameters()):
        assert torch.equal(p1, p0), k


def test_norm_fold_matches_optimizer_norm_pass(cuda):
    """Single process: the clip's norm pass folded into the backward's reduction launch (the
    default) against the optimizer's own norm pass -- the same pre-clip norm up to summation
    order, and the same parameters after 4 graph-replayed AdamW steps."""
    meta, _ = fixtures.load('cmu_cfg3')
    batch = cuda_batch(meta, cuda)
    e1, m1, l1, g1 = _run(lambda: cmu_model(meta, cuda), batch, 4, collective=False, fold_norm=True)
    assert e1._n_ext > 0, 'the norm pass was not folded'
    e0, m0, l0, g0 = _run(lambda: cmu_model(meta, cuda), batch, 4, collective=False, fold_norm=False)
    assert e0._n_ext == 0
    assert float((g1 - g0).abs().max() / g0.abs().max()) < 1e-6, (g1, g0)
    assert float((l1 - l0).abs().max()) <= 1e-6 * float(l0.abs().max()), (l1, l0)
    for (k, p1), (_, p0) in zip(m1.named_parameters(), m0.named_parameters()):
        assert float((p1 - p0).abs().max()) <= 1e-6, k


def _fold_pair(build, steps=4, ptol=1e-6):
    """(engine, model, losses, gnorms) with the norm pass folded and with the optimizer's own pass;
    build(fold_norm) -> (engine, model, step function); ptol: the parameters' absolute agreement
    after the steps"""
    out = []
    for fold in (True, False):
        eng, model, step = build(fold)
        losses, gn = [], []
        for _ in range(steps):
            losses.append(step(eng).clone())
            gn.append(eng.opt.gnorm.clone())
        torch.cuda.synchronize()
        assert (eng._n_ext > 0) == fold, 'fold_norm=%s not honoured' % fold
        out.append((model, torch.cat(losses), torch.cat([g.reshape(1) for g in gn])))
    (m1, l1, g1), (m0, l0, g0) = out
    assert float((g1 - g0).abs().max() / g0.abs().max()) < 1e-6, (g1, g0)
    assert float((l1 - l0).abs().max()) <= 1e-6 * float(l0.abs().max()), (l1, l0)
    for (k, p1), (_, p0) in zip(m1.named_parameters(), m0.named_parameters()):
        e = (p1 - p0).abs()
        assert float(e.max()) <= ptol, (k, float(e.max()), int((e > ptol).sum()), e.numel(), g1, g0)


def test_norm_fold_matches_optimizer_norm_pass_ren_dropout(cuda):
    """Ren-MME at DROP = 0.1 with R-Drop: the shared unify LayerNorm's column sums and the dropout
    epilogues write gradients the folded norm must see; the pre-clip norm at every step and the
    parameters after 4 graph-replayed AdamW steps match the optimizer's own norm pass."""
    from mep_amd import ren_mme
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    meta, _ = fixtures.load('ren_drop_long')
    inputs, labels = fixtures.batch(meta)
    batch = list(ren_mme._pack([t.to(cuda) for t in inputs])) + [labels.to(cuda)]

    def build(fold):
        model = ren_model(meta, cuda, drop=meta['drop']['p'])
        model.train()
        eng = TrainEngine(model, FusedAdamW(model, lr=1e-3), clip=1.0, rdrop=True, graph=True, fold_norm=fold)
        model.mep_runner(cuda).seed_state[0].fill_(31337)
        return eng, model, lambda e: e.step(*batch)
    _fold_pair(build)


def test_norm_fold_matches_optimizer_norm_pass_realformer(cuda):
    """realformer State_Transfer (Adam, position-embedding column sums, the batch-loss column sum
    that is not a gradient): folded norm vs the optimizer's own norm pass over 4 steps.  Adam
    divides each update by its own running magnitude, so the norm's summation-order difference
    (1e-7 relative in the clip coefficient) moves a near-zero-gradient element by up to a few
    1e-6 after 4 steps at lr 1e-3 (1.9e-6 measured on 1 of 1,024 w_qkv elements): 4e-6 here."""
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdam
    from tests.test_gpu_realformer import _batch, _state
    meta, _ = fixtures.load('rf_state_small')
    batch = _batch(meta, cuda)

    def build(fold):
        model = _state(meta, cuda)
        eng = TrainEngine(model, FusedAdam(model, lr=1e-3), clip=1.0, graph=True, fold_norm=fold)
        return eng, model, lambda e: e.step(*batch)
    _fold_pair(build, ptol=4e-6)
