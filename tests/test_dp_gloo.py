"""Data-parallel orchestration of the training engine (engine.TrainEngine) on CPU with the gloo
backend, world_size 2: rank 0's parameters are broadcast once, every rank's
flat gradient buffer is all-reduced (SUM) between backward and optimizer, and the optimizer sees
grad_scale = 1/world, so both ranks end with identical parameters equal to a single-process
AdamW step on the mean gradient (clip after the reduce).

The GPU kernels are replaced by CPU stand-ins (the plan's forward/backward write a rank-dependent
gradient; the optimizer's fused step is the oracle's clip + AdamW with the device hyper-parameters
the engine set), so exactly the host logic runs: broadcast, all-reduce, hyper-parameters.
"""
import os
import socket

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


def _fake_grad(flat, rank):
    g = torch.Generator().manual_seed(100 + rank)
    flat.grad.zero_()
    flat.grad[:flat.n_grad] = torch.randn(flat.n_grad, generator=g) * (1.0 + rank)


class _FakePlan:
    """Stands in for TriModalPlan: forward/backward produce a rank-dependent gradient."""

    def __init__(self, runner, rank):
        self.runner, self.rank = runner, rank
        self.device = runner.device
        self._drop = 0.0
        self.loss = torch.zeros(1)

    def set_dropout(self, p):
        assert p == 0.0

    def set_global_rows(self, n):
        return n

    def forward(self, grad=True, rdrop=False, stream=None):
        pass

    def backward(self, ext_dlogits=None, stream=None):
        _fake_grad(self.runner.flat, self.rank)
        self.loss.fill_(float(self.rank))


def _oracle_step(flat, opt, exp_avg, exp_avg_sq, step):
    """clip_grad_norm_ + AdamW (torch semantics) on grad * grad_scale, from the hyper vector."""
    lr, b1, b2, eps, wd, max_norm, scale = [float(x) for x in opt.hyper[:7]]
    n = flat.n_grad
    g = flat.grad[:n] * scale
    norm = torch.linalg.vector_norm(g)
    coef = min(1.0, max_norm / (float(norm) + 1e-6))
    g = g * coef
    p = flat.buf[:n]
    p.mul_(1 - lr * wd)
    exp_avg[:n].mul_(b1).add_(g, alpha=1 - b1)
    exp_avg_sq[:n].mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    denom = (exp_avg_sq[:n] / bc2).sqrt().add_(eps)
    p.addcdiv_(exp_avg[:n], denom, value=-lr / bc1)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import mep_import
        mep_import.load()
        from mep_amd import cmu_mosei
        from mep_amd.engine import TrainEngine
        from mep_amd.optim import FusedAdamW
        torch.manual_seed(rank)                      # ranks start from DIFFERENT weights
        model = cmu_mosei.Concat_Trans(32, 5, 5, 5, 2, 1, 1)
        opt = FusedAdamW(model, lr=1e-2)
        runner = model.mep_runner('cpu')
        plan = _FakePlan(runner, rank)
        eng = TrainEngine(model, opt, clip=1.0, graph=False)
        assert eng.world == world
        steps = {'n': 0}

        def fused_step(stream=None):
            steps['n'] += 1
            _oracle_step(runner.flat, opt, opt.exp_avg, opt.exp_avg_sq, steps['n'])
        opt.fused_step = fused_step
        start = None
        for _ in range(2):
            eng.step_plan(plan)
            if start is None:
                start = runner.flat.buf.clone()
        out[rank] = dict(buf=runner.flat.buf.clone(), hyper=opt.hyper.clone(), n_grad=runner.flat.n_grad,
                         grad=runner.flat.grad.clone())
    finally:
        dist.destroy_process_group()


def test_engine_dp_world2():
    world = 2
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    r0, r1 = res[0], res[1]
    assert torch.equal(r0['buf'], r1['buf']), 'ranks diverged'
    assert abs(float(r0['hyper'][6]) - 1.0 / world) < 1e-7     # grad_scale = 1/world
    # the reduced gradient is the SUM of both ranks' gradients (scaled in the optimizer)
    import mep_import
    mep_import.load()
    from mep_amd import cmu_mosei
    from mep_amd.flat import FlatParams
    torch.manual_seed(0)
    ref_model = cmu_mosei.Concat_Trans(32, 5, 5, 5, 2, 1, 1)
    spec = ref_model.mep_spec()
    flat = FlatParams(ref_model, 'cpu', no_grad=spec.no_grad_params(), first=spec.bucket_a)   # the runner's layout
    n = flat.n_grad
    grads = []
    for rank in range(world):
        _fake_grad(flat, rank)
        grads.append(flat.grad.clone())
    assert torch.allclose(r0['grad'][:n], (grads[0] + grads[1])[:n])
    # single-process reference: rank 0's initial weights, two steps on the mean gradient
    exp_avg, exp_avg_sq = torch.zeros_like(flat.buf), torch.zeros_like(flat.buf)

    class H:
        hyper = torch.tensor([1e-2, 0.9, 0.999, 1e-8, 1e-2, 1.0, 1.0, 0.0])
    for step in (1, 2):
        flat.grad.copy_((grads[0] + grads[1]) / world)
        _oracle_step(flat, H, exp_avg, exp_avg_sq, step)
    assert torch.allclose(r0['buf'][:n], flat.buf[:n], rtol=1e-5, atol=1e-7)


if __name__ == '__main__':
    pytest.main([__file__, '-q'])
