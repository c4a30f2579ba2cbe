"""Throughput of the cmu-mosei tri-modal training step on MI355X (BASELINE.json metric).

Workload (BASELINE cfg3 / cfg4): Concat_Trans (D=96, H=6, n_layers=1, 7 classes), B=64 utterance
pairs per GPU, T=50 for text (d=300), visual (d=35) and audio (d=74); one step = forward of both
encoders + head + circle loss + backward + clip_grad_norm_(1.0) + AdamW (lr 1e-3) [+ RCCL
all-reduce of the flat gradient when N > 1].  Synthetic N(0,1) features, all-ones masks,
Bernoulli(0.3) labels, random-init weights; inputs resident in HBM before the timed region.
Arithmetic: fp32 end to end (the reference has no AMP; fp32 keeps the 1e-4 logits parity).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)
Rank 0 prints one JSON line.
"""
import argparse
import glob
import json
import os
import re
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()

METRIC = 'utterances/sec fwd+bwd, CMU-MOSEI tri-modal B=64 T=50, 1/2/4/8 MI355X'
B, T, D, H, NL = 64, 50, 96, 6, 1
DIMS = (300, 35, 74)


class LaunchTimer:
    """HIP events around every libmep launch of an eager step, on the launching stream (the
    backward's side-stream launches included)."""

    def __init__(self):
        self.ev = []

    def begin(self, name, stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream if stream is not None else torch.cuda.current_stream())
        self.ev.append([name, e, None])

    def end(self, name, stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream if stream is not None else torch.cuda.current_stream())
        self.ev[-1][2] = e

    def totals(self):
        torch.cuda.synchronize()
        out = {}
        for name, a, b in self.ev:
            t, n = out.get(name, (0.0, 0))
            out[name] = (t + a.elapsed_time(b) / 1e3, n + 1)
        return out


# launch name -> kernel symbol prefix in the rocprofv3 summaries (scripts/parse_prof.py)
KERNEL_OF = {'mep_attn_bwd': 'k_attn_bwd', 'mep_attn_fwd': 'k_attn_fwd', 'mep_block_epi_fwd': 'k_epi_fwd',
             'mep_block_epi_bwd': 'k_epi_bwd', 'mep_wgrad': 'k_wgrad', 'mep_unify': 'k_unify',
             'mep_pool_fwd': 'k_pool_fwd', 'mep_pool_bwd': 'k_pool_bwd'}


def pmc_traffic(launch):
    """(HBM bytes per dispatch, source file) of the kernel behind `launch` from the newest
    committed PMC pass (profiles/r<round>_v<n>_pmc.json: (2 FETCH_SIZE + WRITE_SIZE) x 1024,
    the gfx950 correction of MI355X_MICROARCH.md section HBM), or (None, None)."""
    def key(f):
        return [int(x) for x in re.findall(r'\d+', os.path.basename(f))]
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_v*_pmc.json')), key=key)
    prefix = KERNEL_OF.get(launch)
    if not files or prefix is None:
        return None, None
    for k, v in json.load(open(files[-1])).items():
        if k.startswith(prefix) and 'hbm_bytes_per_dispatch' in v:
            return int(v['hbm_bytes_per_dispatch']), os.path.relpath(files[-1], ROOT)
    return None, None


def synth_batch(rank, device):
    rng = np.random.default_rng(20261015 + rank)
    f = lambda d: torch.from_numpy(rng.standard_normal((B, 2, T, d), dtype=np.float32)).to(device)  # noqa: E731
    l, v, a = (f(d) for d in DIMS)
    m = torch.ones(B, 2, T, device=device)
    labels = torch.from_numpy((rng.random((B, 7)) < 0.3).astype(np.int64)).to(device)
    return l, v, a, m, m.clone(), m.clone(), labels


def cpu_baseline(budget_s=12.0):
    """The CPU oracle (repo restatement of the reference path, fp32 PyTorch CPU) on the same
    workload: fwd+bwd+clip+AdamW at B=64, T=50, timed for a bounded number of steps."""
    from oracle import cmu_mosei as ocmu
    from oracle import common
    from tests.golden import specs
    from mep_amd import cmu_mosei
    m = cmu_mosei.Concat_Trans(dim=D, l_len=T, v_len=T, a_len=T, n_heads=H, n_layers=NL, ffn=1)
    shapes = {k: list(v.shape) for k, v in m.state_dict().items()}
    P = {k: torch.tensor(v, requires_grad=True) for k, v in specs.param_values(shapes, 1).items()}
    opt = common.AdamState(P.values(), lr=1e-3, weight_decay=0.01)
    batch = [torch.from_numpy(x) for x in specs.cmu_batch(seed=5, B=B, T=T, no_name_rows=(), full_masks=True)]
    ocmu.train_step(P, opt, batch, H, NL)       # warmup
    n, t0 = 0, time.perf_counter()
    while True:
        ocmu.train_step(P, opt, batch, H, NL)
        n += 1
        el = time.perf_counter() - t0
        if (n >= 3 and el >= budget_s) or n >= 200:
            break
    return dict(value=round(B * n / el, 2), unit='utt/s', cores=torch.get_num_threads(), kind='port',
                sample='%d steps of B=64,T=50 Concat_Trans fwd+bwd+clip+AdamW (oracle, fp32 CPU, %d threads)'
                       % (n, torch.get_num_threads()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--cpu-budget', type=float, default=12.0)
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)

    from mep_amd import cmu_mosei, roofline
    from mep_amd import _lib
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW

    torch.manual_seed(0)
    model = cmu_mosei.Concat_Trans(dim=D, l_len=T, v_len=T, a_len=T, n_heads=H, n_layers=NL, ffn=1).to(dev).train()
    opt = FusedAdamW(model, lr=1e-3)
    eng = TrainEngine(model, opt, clip=1.0, graph=not args.no_graph)
    batch = synth_batch(rank, dev)
    plan = model.mep_runner(dev).plan(B, (T, T, T))
    plan.set_inputs(*batch)

    for _ in range(args.warmup):
        eng.step_plan(plan)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step_plan(plan)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    loss = float(plan.loss.item())

    # per-launch HIP-event timing of eager steps -> dominant kernel roofline
    timer = LaunchTimer()
    reps = 20
    eng_eager = TrainEngine(model, opt, clip=1.0, graph=False)
    _lib.TIMER = timer
    for _ in range(reps):
        eng_eager.step_plan(plan)
    _lib.TIMER = None
    tot = timer.totals()
    costs = roofline.launch_costs(plan)
    per_kernel = {k: dict(ms_per_step=round(t / reps * 1e3, 4), launches_per_step=n // reps)
                  for k, (t, n) in sorted(tot.items(), key=lambda kv: -kv[1][0])}
    dom = max((k for k in tot if k in costs), key=lambda k: tot[k][0])
    t_dom, n_dom = tot[dom]
    per_launch_s = t_dom / n_dom
    launches_per_step = n_dom // reps
    flops, nbytes = costs[dom]
    rl = roofline.roofline_entry(dom, flops / launches_per_step, nbytes / launches_per_step, per_launch_s)
    rl['traffic'], rl['traffic_source'] = pmc_traffic(dom)
    rl['avg_launch_us'] = round(per_launch_s * 1e6, 2)

    out = {
        'metric': METRIC,
        'value': round(B * world * args.steps / el, 2),
        'unit': 'utt/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(el / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'fp32',
        'data': 'synthetic N(0,1) features, all-ones masks, Bernoulli(0.3) labels, random-init weights',
        'config': {'workload': 'cmu-mosei Concat_Trans train step (fwd+bwd+clip+AdamW), BASELINE cfg3/cfg4',
                   'global_batch': B * world, 'per_gpu_batch': B, 'seq_len': T, 'dims': list(DIMS),
                   'D': D, 'heads': H, 'n_layers': NL, 'parallelism': 'dp%d' % world,
                   'graph': not args.no_graph},
        'loss': round(loss, 6),
        'roofline': rl,
        'kernels': per_kernel,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(args.cpu_budget)
        out['gpu_vs_cpu'] = round(out['value'] / out['cpu_baseline']['value'], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
