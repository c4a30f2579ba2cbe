"""Data-parallel epoch plumbing (mep_amd.dp) on CPU with gloo, world_size 2:

* sharding: every rank sees rank 0's shuffled order; each global batch is split into contiguous
  per-rank units (Ren-MME duplicate pairs never straddle ranks, cmu-mosei / realformer units are
  whole pairs / groups); the ragged last global batch may leave a rank an empty share;
* train(): each rank steps on its share with ``global_rows`` of the whole global batch (an empty
  share still joins the step), and the epoch loss is the global one on every rank -- equal to a
  single process's mean over the same global batches;
* run(): the plateau scheduler, early stopping and checkpoint choice see the same global valid
  loss on every rank; only rank 0 writes the log and the checkpoints.

The GPU engine is replaced by a stand-in whose step returns the rank's share of a per-row loss
(each row's loss is a function of its label), so exactly the host logic runs here; the GPU
equivalence of a sharded step and the 1-rank step on the concatenated batch is
tests/test_gpu_dp.py.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _row_loss(label_row):
    return 0.1 + float(np.asarray(label_row, np.float64).sum()) * 0.37


def _spawn(fn, world=2):
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_entry, args=(fn, world, port, out), nprocs=world, join=True)
        return dict(out)


def _entry(rank, fn, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import mep_import
        mep_import.load()
        out[rank] = fn(rank, world)
    finally:
        dist.destroy_process_group()


# ------------------------------------------------------------------------------ sharding
def _shard_worker(rank, world):
    from mep_amd import dp
    random.seed(100 + rank)                 # ranks' own RNG states differ on purpose
    names = ['u%d' % i for i in range(23)]
    dp.shared_shuffle(names)
    # Ren-MME style: every sample twice, global batches of 2 * 5 rows
    rows = [(n, k) for n in names for k in (0, 1)]
    glob = [rows[i:i + 10] for i in range(0, len(rows), 10)]
    shards = [(list(s), s.global_rows) for s in dp.shard_batches(iter(glob), unit=2)]
    row0s = [s.row0 for s in dp.shard_batches(iter(glob), unit=2)]
    return dict(order=names, shards=shards, row0s=row0s)


def test_shards_world2():
    res = _spawn(_shard_worker)
    assert res[0]['order'] == res[1]['order'], 'ranks must share rank 0 shuffled order'
    s0, s1 = res[0]['shards'], res[1]['shards']
    assert len(s0) == len(s1)
    for (a, ga), (b, gb) in zip(s0, s1):
        assert ga == gb == len(a) + len(b)
        for part in (a, b):                  # duplicate pairs stay together
            assert len(part) % 2 == 0
            assert all(part[i][0] == part[i + 1][0] for i in range(0, len(part), 2))
    # the shares are the contiguous halves of each global batch, in order
    order = res[0]['order']
    rows = [(n, k) for n in order for k in (0, 1)]
    flat = [r for (a, _), (b, _) in zip(s0, s1) for r in list(a) + list(b)]
    assert [tuple(r) for r in flat] == rows
    assert s1[-1][0] == [] or len(s1[-1][0]) < len(s0[-1][0])   # ragged tail: rank 1 has less
    # row0: global index of each share's first row (rank 1 starts after rank 0's whole share)
    assert all(r == 0 for r in res[0]['row0s'])
    assert [r for r in res[1]['row0s']] == [len(a) for (a, _) in s0]


# ------------------------------------------------------------------------------ train / run
class _FakeEngine:
    """step(): the rank's share of the global-batch mean of _row_loss; step_empty(): 0."""

    def __init__(self):
        self.calls = []
        self.row0s = []

    def step(self, *cols, global_rows=None, row0=0):
        label = cols[6]
        n = global_rows if global_rows is not None else label.shape[0]
        self.calls.append(('step', int(label.shape[0]), global_rows))
        self.row0s.append(row0)
        return torch.tensor([sum(_row_loss(r) for r in label.tolist()) / n], dtype=torch.float32)

    def step_empty(self, device):
        self.calls.append(('empty', 0, None))
        return torch.zeros(1)


def _batches(order, per_rank, world):
    """Global batches of (prev, cur) 'rows' as the reference's data_loader yields them."""
    rng = np.random.default_rng(0)
    labels = {n: (rng.random(7) < 0.4).astype(np.int64) for n in order}
    rows = [(np.zeros(1), np.zeros(1), np.zeros(1), np.zeros(1), np.zeros(1), np.zeros(1), labels[n]) for n in order]
    step = per_rank * world
    return [rows[i:i + step] for i in range(0, len(rows), step)]


def _train_worker(rank, world):
    from mep_amd import cmu_mosei, dp, engine, optim
    eng = _FakeEngine()
    cmu_mosei._to_device = lambda batch, device: [torch.from_numpy(np.stack(c)) for c in zip(*batch)]
    engine.engine_for = lambda *a, **k: eng
    order = ['u%d' % i for i in range(13)]
    glob = _batches(order, 3, world)
    model = cmu_mosei.Concat_Trans(32, 5, 5, 5, 2, 1, 1)
    opt = optim.FusedAdamW(model, lr=1e-3)
    loss = cmu_mosei.train(model, dp.shard_batches(iter(glob), per_rank=3), opt, device='cpu')
    return dict(loss=loss, calls=eng.calls, row0s=eng.row0s)


def test_train_epoch_loss_is_global_world2():
    res = _spawn(_train_worker)
    assert res[0]['loss'] == res[1]['loss']
    # single-process value: mean over global batches of the global-batch mean row loss
    order = ['u%d' % i for i in range(13)]
    glob = _batches(order, 3, 2)
    want = np.mean([np.mean([_row_loss(r[6]) for r in g]) for g in glob])
    assert abs(res[0]['loss'] - want) < 1e-6
    # 13 pairs, 6 per global batch: the last global batch has 1 pair -> rank 1's share is empty
    assert res[1]['calls'][-1][0] == 'empty'
    assert res[0]['calls'][-1] == ('step', 1, 1)
    assert all(c[2] == 6 for c in res[0]['calls'][:-1])
    assert all(r == 0 for r in res[0]['row0s']) and all(r == 3 for r in res[1]['row0s'])


def _run_worker(rank, world, tmp):
    from mep_amd import cmu_mosei, dp, engine
    eng = _FakeEngine()
    cmu_mosei._to_device = lambda batch, device: [torch.from_numpy(np.stack(c)) for c in zip(*batch)]
    engine.engine_for = lambda *a, **k: eng
    # valid: the "logits" are the labels, the loss a rank-dependent function of them, so the
    # ranks' local valid sums differ and only the all-reduced global value can agree
    cmu_mosei.multi_circle_loss = lambda logits, label: label.double().sum(1) * 0.3 + 0.2
    model = cmu_mosei.Concat_Trans(32, 5, 5, 5, 2, 1, 1)
    model.forward = lambda l, v, a, lm, vm, am: None
    epochs = iter(range(100))
    import torch.optim.lr_scheduler as sched
    seen = []

    class Recorded(sched.ReduceLROnPlateau):
        def step(self, metrics):
            super().step(metrics)
            seen.append((float(metrics), float(self.optimizer.param_groups[0]['lr'])))
    sched.ReduceLROnPlateau = Recorded

    def data_loader(names, label_dict, batch_size):
        e = next(epochs)
        rng = np.random.default_rng(e // 2)        # valid/train of one epoch share a seed
        rows = [(np.zeros(1),) * 6 + ((rng.random(7) < 0.2 + 0.05 * (e % 7)).astype(np.int64),) for _ in names]
        glob = [rows[i:i + 4 * dp.world()] for i in range(0, len(rows), 4 * dp.world())]
        return dp.shard_batches(iter(glob), per_rank=4)
    cmu_mosei.run(model, ['a'] * 11, ['b'] * 9, {}, 4, 1e-3, 12, 'dp', data_loader=data_loader, log_dir=tmp,
                  device='cpu')
    return dict(files=sorted(os.listdir(tmp)) if rank == 0 else [f for f in os.listdir(tmp) if f.endswith('.pt')],
                seen=seen)


def _run_entry(rank, world, dirs):
    return _run_worker(rank, world, dirs[rank])


def test_run_decisions_world2(tmp_path):
    import functools
    dirs = [str(tmp_path / 'r0'), str(tmp_path / 'r1')]
    for d in dirs:
        os.makedirs(d)
    res = _spawn(functools.partial(_run_entry, dirs=dirs))
    assert res[1]['files'] == [], 'rank 1 must not write checkpoints'
    assert not os.listdir(dirs[1]), 'rank 1 must not write the log either'
    assert any(f.endswith('.pt') for f in res[0]['files']) and 'dp.txt' in res[0]['files']
    # identical global valid losses -> identical plateau / early-stop decisions on both ranks
    assert res[0]['seen'] == res[1]['seen'] and len(res[0]['seen']) >= 2
    assert len({lr for _, lr in res[0]['seen']}) >= 2, 'the plateau scheduler should have fired'
