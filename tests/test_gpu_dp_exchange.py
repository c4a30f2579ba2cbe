"""The bucketed data-parallel gradient exchange with a real SUM, on one GPU (SURVEY.md 8(e);
reference step cmu-mosei/run.py:364-369: backward, clip_grad_norm_, AdamW.step).

A world-1 ``nccl`` (= RCCL) group puts TrainEngine on its production DP path: the flat gradient in
two buckets, bucket A's all-reduce issued on a side stream from inside ``backward_bucketed`` while
the last attention backward and the unify weight gradients still run, bucket B's after them, all
of it captured in the step's hipGraph from the second step on.  ``dist.all_reduce`` is replaced by
a stand-in for a SUM over TWO IDENTICAL RANKS: it records the range it was given, copies the
buffer as it is at call time (on the caller's stream, so under capture the copy is replayed too)
and multiplies it by 2 in place.  The engine runs as rank 0 of 2 with ``global_rows = 2 B`` (each
rank's loss scaled to its part of the global mean), so a real 2-rank run on the batch and itself
would compute exactly this.

Checked, eager and under graph capture:
  * the recorded ranges partition [0, n_grad) exactly once per step;
  * bucket A as the collective sees it (the snapshot) is final: times 2 it equals, bit for bit,
    the gradient of the engine without any collective at the same step, taken right before its
    optimizer (1/(2B) loss scale times the SUM's 2 is exact in fp32), so no launch of the backward
    was still writing it -- no readiness race -- and bucket B likewise;
  * the post-SUM gradient (before clip + AdamW, which scale the gradient in place as
    clip_grad_norm_ does), loss and post-step parameters equal the no-collective engine's bit for
    bit at every step;
  * the post-step parameters equal a one-rank step on the batch concatenated with itself (2 B rows;
    summation order differs, so within fp32 noise).
"""
import socket

import pytest
import torch
import torch.distributed as dist

from tests.golden import fixtures
from tests.gpu_util import assert_close, cmu_model, cuda_batch, ren_model

pytestmark = pytest.mark.gpu

STEPS = 3
LR = 1e-3


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


class TwoRankSum:
    """dist.all_reduce(SUM) over two ranks holding the same gradient: x -> 2 x, recording each
    call's (offset, numel) in the flat gradient and a copy of the buffer at call time."""

    def __init__(self, grad):
        self.grad = grad
        self.calls = []
        self.snaps = {}

    def __call__(self, t, op=dist.ReduceOp.SUM, group=None, async_op=False):
        assert op == dist.ReduceOp.SUM and not async_op
        assert t.dtype == torch.float32 and t.is_contiguous()
        base = self.grad.data_ptr()
        assert base <= t.data_ptr() < base + 4 * self.grad.numel(), 'all-reduce of a buffer outside flat.grad'
        key = ((t.data_ptr() - base) // 4, t.numel())
        snap = self.snaps.get(key)
        if snap is None:                 # first (eager) step: capture reuses the buffer
            assert not torch.cuda.is_current_stream_capturing()
            snap = self.snaps[key] = torch.empty_like(t)
        snap.copy_(t)                    # on the caller's stream: bucket A's side stream
        t.mul_(2.0)
        self.calls.append(key)


def _engine(model, collective, graph):
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    model.train()
    opt = FusedAdamW(model, lr=LR)
    # the collective engine keeps the optimizer's own norm pass (the norm follows the SUM); the
    # engines it is compared with bit for bit do too
    eng = TrainEngine(model, opt, clip=1.0, rdrop=False, graph=graph, collective=collective, fold_norm=False)
    # the flat gradient as the optimizer receives it (clip + AdamW then scale it in place), copied
    # on the step's stream -- inside the captured graph too, so a replay refreshes the copy
    eng.pre_opt = None
    run_opt = eng._opt

    def opt_with_copy():
        flat = model.mep_runner(next(model.parameters()).device).flat
        if eng.pre_opt is None:
            assert not torch.cuda.is_current_stream_capturing()
            eng.pre_opt = torch.empty_like(flat.grad[:flat.n_grad])
        eng.pre_opt.copy_(flat.grad[:flat.n_grad])
        run_opt()
    eng._opt = opt_with_copy
    return eng


def _double(batch):
    out = []
    for t in batch:
        if isinstance(t, (tuple, list)):
            out.append(type(t)(torch.cat([x, x]) for x in t))
        else:
            out.append(torch.cat([t, t]))
    return out


def _params(model):
    return {k: p.detach().clone() for k, p in model.named_parameters()}


def _exchange_case(model_fn, batch, B, graph, monkeypatch, rdrop=False, doubled=True):
    # -- the DP engine: rank 0 of two identical ranks
    mc = model_fn()
    ec = _engine(mc, True, graph)
    ec.rdrop = rdrop
    assert ec.collective and ec.overlap, 'the bucketed exchange path is not selected'
    ec.world = 2                      # rank 0 of 2: loss scaled by 1 / global_rows, plain SUM into the optimizer
    runner = mc.mep_runner(batch[-1].device)
    fl = runner.flat
    assert 0 < fl.split < fl.n_grad
    fake = TwoRankSum(fl.grad)
    monkeypatch.setattr(dist, 'all_reduce', fake)
    c_steps = []
    for k in range(STEPS):
        fake.calls = []
        loss = ec.step(*batch, global_rows=2 * B, row0=0).clone()
        torch.cuda.synchronize()
        # one call per bucket per executed or captured body: the first graph step runs eagerly and
        # then captures (host calls twice); its replays make no host call
        want = [(0, fl.split), (fl.split, fl.n_grad - fl.split)]
        if graph:
            want = sorted(want * 2) if k == 0 else []
        assert sorted(fake.calls) == want, ('step %d' % k, fake.calls, fl.split, fl.n_grad)
        snaps = {key: s.clone() for key, s in fake.snaps.items()}
        c_steps.append((loss, ec.pre_opt.clone(), snaps, _params(mc)))
    if graph:
        assert ec.capture_allreduce and all(b is None for (_, b) in ec._graphs.values()), \
            'the all-reduce was not captured in the step graph'
    monkeypatch.undo()

    # -- the engine without a collective, same batch
    mr = model_fn()
    er = _engine(mr, False, graph)
    er.rdrop = rdrop
    flr = mr.mep_runner(batch[-1].device).flat
    assert (flr.split, flr.n_grad) == (fl.split, fl.n_grad)
    for k in range(STEPS):
        loss = er.step(*batch).clone()
        torch.cuda.synchronize()
        lc, gc, snaps, pc = c_steps[k]
        gr = er.pre_opt
        a = snaps[(0, fl.split)]
        b = snaps[(fl.split, fl.n_grad - fl.split)]
        assert torch.equal(2.0 * a, gr[:fl.split]), 'step %d: bucket A was not final at its all-reduce' % k
        assert torch.equal(2.0 * b, gr[fl.split:]), 'step %d: bucket B was not final at its all-reduce' % k
        assert torch.equal(gc, gr), 'step %d: post-SUM gradient' % k
        assert torch.equal(2.0 * lc, loss), ('step %d: loss' % k, lc, loss)
        pr = _params(mr)
        for name in pr:
            assert torch.equal(pc[name], pr[name]), 'step %d: %s' % (k, name)

    if not doubled:
        return
    # -- one rank, the batch concatenated with itself (2 B rows), one step
    md = model_fn()
    ed = _engine(md, False, False)
    ed.rdrop = rdrop
    ed.step(*_double(batch))
    torch.cuda.synchronize()
    fld = md.mep_runner(batch[-1].device).flat
    gd = ed.pre_opt
    _, gc1, _, pc1 = c_steps[0]
    assert_close(gc1, gd, 1e-4, 1e-5, 'DP gradient vs the doubled batch')
    gfull = torch.zeros_like(fld.grad)
    gfull[:fld.n_grad] = gd
    gd_view = {n: fld.view(gfull, n) for n in fld.names if fld.has_grad[n]}
    for name, p in md.named_parameters():
        # the suite's post-step standard (gpu_util.check_post_params): atol 2e-5, and |delta| <= 2 lr
        # where the gradient is at rounding-noise level (|g| < 1e-6: Adam's first step follows
        # its last ulps)
        err = (pc1[name] - p.detach()).abs()
        tol = torch.full_like(err, 2e-5)
        if name in gd_view:
            tol = torch.where(gd_view[name].abs() < 1e-6, torch.full_like(err, 2 * LR + 2e-5), tol)
        assert bool((err <= tol).all()), (name, float(err.max()))


@pytest.mark.parametrize('graph', [False, True], ids=['eager', 'graph'])
def test_dp_exchange_two_rank_sum_cmu_cfg3(nccl_world1, cuda, graph, monkeypatch):
    """BASELINE cfg3 (B = 64, T = 50, Concat_Trans): the cfg4 data-parallel step on one GPU."""
    meta, _ = fixtures.load('cmu_cfg3')
    batch = cuda_batch(meta, cuda)
    _exchange_case(lambda: cmu_model(meta, cuda), batch, batch[-1].shape[0], graph, monkeypatch)


@pytest.mark.parametrize('graph', [False, True], ids=['eager', 'graph'])
def test_dp_exchange_two_rank_sum_cmu_cfg3_bf16(nccl_world1, cuda, graph, monkeypatch):
    """The same exchange on the bf16 path (the bench's default precision for cfg3 / cfg4): bf16
    activations, fp32 flat gradient and optimizer.  Every bit-for-bit check holds as on the fp32
    path (the power-of-two loss scale and the SUM's 2 are exact); the doubled-batch comparison is
    left to the fp32 cases (2 B rows change the weight-gradient chunking, whose bf16 rounding then
    differs by more than the fp32 post-step tolerance)."""
    meta, _ = fixtures.load('cmu_cfg3')
    batch = cuda_batch(meta, cuda)

    def model():
        m = cmu_model(meta, cuda)
        m.mep_precision = 'bf16'
        return m
    _exchange_case(model, batch, batch[-1].shape[0], graph, monkeypatch, doubled=False)


@pytest.mark.parametrize('graph', [False, True], ids=['eager', 'graph'])
def test_dp_exchange_two_rank_sum_ren(nccl_world1, cuda, graph, monkeypatch):
    """Ren-MME (D = 128, Tk = 80, shared unify LayerNorm in bucket B) with the R-Drop head: the
    KL's global pair count doubles with the global rows."""
    from mep_amd import ren_mme
    meta, _ = fixtures.load('ren_drop_long')
    inputs, labels = fixtures.batch(meta)
    batch = list(ren_mme._pack([t.to(cuda) for t in inputs])) + [labels.to(cuda)]
    B = labels.shape[0]
    assert B % 2 == 0
    _exchange_case(lambda: ren_model(meta, cuda, drop=0.0), batch, B, graph, monkeypatch, rdrop=True)
