"""Two real data-parallel ranks on the GPU: two processes, each running the full
HIP training step on its share of a global batch and exchanging the flat gradient through
torch.distributed, checked against the reference's single-process step.

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), and the GPU boxes here have one, so
the ranks exchange over gloo on device tensors: everything else is the production data-parallel
path -- the real plans and kernels, the rank-0 parameter broadcast, the 1/B_global loss scale of
unequal shares (5 + 3 rows), the host-side all-reduce between the engine's two graphs, the
optimizer's own norm pass after the SUM.  Only the captured RCCL collective (test_gpu_rccl.py,
world 1; test_gpu_dp_exchange.py, a recording two-rank SUM) is not on this path.

Checks, cmu_cfg1 (B = 8, T = 50, D = 96, ragged masks):
  * step 1 on both ranks equals the reference's full-batch step: the sum of the ranks' losses,
    the global gradient norm and every post-AdamW parameter (gpu_util.check_post_params);
  * the ranks hold bit-identical parameters after every step (eager first step, then the
    captured graphs with the host all-reduce between them);
  * step 2 agrees with a single-process engine on the whole batch.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CUT = 5          # rank 0 takes rows [0, 5), rank 1 rows [5, 8)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import mep_import
        mep_import.load()
        from mep_amd.engine import TrainEngine
        from mep_amd.optim import FusedAdamW
        from tests.golden import fixtures
        from tests.gpu_util import cmu_model, cuda_batch
        dev = torch.device('cuda:0')
        meta, _ = fixtures.load('cmu_cfg1')
        torch.manual_seed(rank)
        model = cmu_model(meta, dev).train()
        if rank == 1:                        # rank 0's weights must reach every rank
            with torch.no_grad():
                for p in model.parameters():
                    p.add_(0.25)
        opt = FusedAdamW(model, lr=1e-3)
        eng = TrainEngine(model, opt, clip=1.0, graph=True)
        assert eng.world == world and eng.collective and not eng.capture_allreduce
        full = cuda_batch(meta, dev)
        lo, hi = (0, CUT) if rank == 0 else (CUT, full[-1].shape[0])
        share = [t[lo:hi].contiguous() for t in full]
        n = full[-1].shape[0]
        res = {}
        for step in (1, 2):
            loss = float(eng.step(*share, global_rows=n, row0=lo).item())
            torch.cuda.synchronize()
            res[step] = dict(loss=loss, gnorm=float(opt.gnorm.item()),
                             params={k: p.detach().cpu().clone() for k, p in model.named_parameters()})
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_reference_step(cuda):
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    from tests.golden import fixtures
    from tests.gpu_util import assert_close, check_post_params, cmu_model, cuda_batch
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    with ctx.Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_worker, args=(world, port, out), nprocs=world, join=True, start_method='spawn')
        res = {r: out[r] for r in range(world)}
    meta, gold = fixtures.load('cmu_cfg1')
    # step 1: the reference's full-batch step
    s1 = [res[r][1] for r in range(world)]
    assert_close(s1[0]['loss'] + s1[1]['loss'], gold['loss'], 1e-5, 0, 'loss (sum of shares)')
    assert_close(s1[0]['gnorm'], gold['gnorm'], 1e-4, 0, 'gnorm')
    model = cmu_model(meta, cuda)
    for r in range(world):
        with torch.no_grad():
            for k, p in model.named_parameters():
                p.copy_(s1[r]['params'][k])
        check_post_params(model, meta, gold)
    for step in (1, 2):
        for k in s1[0]['params']:
            assert torch.equal(res[0][step]['params'][k], res[1][step]['params'][k]), (step, k)
    # step 2 (graph replay + host all-reduce) against one process on the whole batch
    ref = cmu_model(meta, cuda).train()
    opt = FusedAdamW(ref, lr=1e-3)
    eng = TrainEngine(ref, opt, clip=1.0, graph=False)
    batch = cuda_batch(meta, cuda)
    for _ in range(2):
        eng.step(*batch)
    torch.cuda.synchronize()
    lr = 1e-3
    n_off = n_all = 0
    for k, p in ref.named_parameters():
        err = (res[0][2]['params'][k].double() - p.detach().cpu().double()).abs()
        assert float(err.max()) <= 4.0 * lr + 1e-5, k       # two steps of at most lr each way
        n_off += int((err > 2e-5).sum())
        n_all += err.numel()
    assert n_off <= max(4, n_all // 1000), (n_off, n_all)
