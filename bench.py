"""Throughput of the tri-modal training path on MI355X (BASELINE.json metric and configs).

Default workload (BASELINE cfg3 / cfg4): cmu-mosei Concat_Trans (D=96, H=6, n_layers=1, 7 classes),
B=64 utterance pairs per GPU, T=50 for text (d=300), visual (d=35) and audio (d=74); one step =
forward of both encoders + head + circle loss + backward + clip_grad_norm_(1.0) + AdamW (lr 1e-3)
[+ RCCL all-reduce of the flat gradient when N > 1].  Synthetic N(0,1) features, all-ones masks,
Bernoulli(0.3) labels, random-init weights; inputs resident in HBM before the timed region.

Arithmetic of the headline line: fp32, the reference's own precision (cmu-mosei/run.py:360-369 has
no AMP) -- fp32 storage, softmax, LayerNorm and accumulation; the products run on the matrix cores
as fp32 operands split into bf16 parts, within the 1e-4 logits parity of the
reference.  BASELINE.json names bf16 for cfg3 / cfg5: that path (bf16 operands and activation
storage, fp32 accumulation, statistics, loss, gradients and AdamW; held to torch.autocast(bf16)'s
own error, tests/test_gpu_bf16.py) is timed in the same run and nested as "bf16".

Per-kernel times ("kernels", "roofline*") are in-step device times
(time_launches: real-time-counter stamps around each launch of a captured step), so they
exclude host submission gaps and sum to at most the step time.
"hbm_measured" is the box's measured HBM peak (mep_hbm_probe) beside the 8 TB/s spec.

    python bench.py [--gpus N --steps K --warmup W]        BASELINE cfg3 (cfg4 with N > 1), fp32 + bf16
    python bench.py --config cfg2 | cfg5 | rfstate        the other workloads
    python bench.py --dtype bf16                          the bf16 path as the headline line
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)
Rank 0 prints one JSON line.  `--gpus N` without WORLD_SIZE starts the N ranks itself
(launch_ranks: torch.distributed.run as a child process); with WORLD_SIZE set it must equal N, and
a node with fewer than N GPUs is refused (exit 2) rather than reported as a smaller run.
"""
import argparse
import glob
import json
import os
import platform
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


class StampTimer:
    """_lib.TIMER hook: a mep_stamp kernel (the device's real-time counter, stored when it starts)
    before and after every entry-point call, on the call's stream."""

    def __init__(self, slots):
        self.slots, self.names, self.n = slots, [], 0

    def _stamp(self, stream):
        import ctypes
        from mep_amd import _lib
        assert self.n < self.slots.numel()
        _lib.check(_lib.lib().mep_stamp(ctypes.c_void_p(self.slots.data_ptr()), self.n, _lib.stream_ptr(stream)),
                   'mep_stamp')
        self.n += 1

    def begin(self, name, stream=None):
        self.names.append(name)
        self._stamp(stream)

    def end(self, name, stream=None):
        self._stamp(stream)


def time_launches(work, reps=41):
    """Device time of every libmep launch of a training step, where it runs in the step.

    The step body (forward, backward, clip + optimizer) is captured into a graph with a mep_stamp
    kernel before and after every launch (a one-wave kernel storing the 100-MHz real-time counter
    as it starts; graph kernels run back to back) and replayed `reps` times.  A launch's time is
    the interval between its two stamps minus the interval of two stamps with nothing between
    them (16 such pairs at the head of the same graph): the launch's execution plus its dispatch, in
    the step -- after the same producers, with the same cache contents -- which is what a
    rocprofv3 trace of a graph step reports per kernel (a kernel's start there is its
    predecessor's end).  HIP events cannot give this on ROCm: timing markers add ~3-5 us to every
    bracketed launch (hipExtLaunchKernel's events included), external event nodes are refused
    under capture, and a launch replayed alone re-reads what its previous replay left in the
    256-MB Infinity Cache (up to ~15% fast).  The replays update the model: this runs after the
    timed region and the loss readout.

    Returns ({launch name: (seconds per step over its launches, launches per step)}, method)."""
    import ctypes
    from mep_amd import _lib
    L = _lib.lib()
    khz = L.mep_stamp_khz()
    assert khz > 0, _lib.last_error()
    tick = 1.0 / (khz * 1e3)
    dev = work.plan.device if hasattr(work.plan, 'device') else torch.device('cuda', torch.cuda.current_device())
    slots = torch.zeros(4096, dtype=torch.int64, device=dev)

    def capture(body):
        timer = StampTimer(slots)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        _lib.TIMER = timer
        try:
            with torch.cuda.graph(g):
                body()
        finally:
            _lib.TIMER = None
        return g, timer

    def intervals(g, n):
        """per stamp pair, the median over `reps` replays (robust to a replay caught by a clock or
        queue hiccup)"""
        for _ in range(3):
            g.replay()
        runs = []
        for _ in range(reps):
            g.replay()
            torch.cuda.synchronize()
            s = slots[:n].cpu().double().reshape(-1, 2)
            runs.append((s[:, 1] - s[:, 0]) * tick)
        return torch.stack(runs).median(dim=0).values

    def body():
        # calibration pairs first, in the same graph: two adjacent stamps under the step's own
        # clocks and queue state
        for _ in range(CAL):
            _lib.TIMER.begin('stamp pair')
            _lib.TIMER.end('stamp pair')
        work.step_body()
    CAL = 16
    g, timer = capture(body)
    iv = intervals(g, timer.n)
    overhead = float(iv[:CAL].mean())
    per = iv[CAL:] - overhead
    timer.names = timer.names[CAL:]
    del g
    tot = {}
    for name, t in zip(timer.names, per.tolist()):
        s0, c = tot.get(name, (0.0, 0))
        tot[name] = (s0 + t, c + 1)
    method = ('in-step: real-time-counter stamps around each launch of a captured step, median of %d replays, '
              'minus the %.2f-us interval of two adjacent stamps' % (reps, overhead * 1e6))
    return tot, method


def hbm_probe(dev, gib=2):
    """Measured HBM peaks (GB/s) of mep_hbm_probe's copy / read / write streams over 2-GiB
    buffers (8x the 256-MB Infinity Cache), best over a few grid sizes (the
    vendor spec and a measured copy-kernel peak, both reported)."""
    import ctypes
    from mep_amd import _lib
    n16 = (gib << 30) // 16
    src = torch.ones(n16 * 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    out = {}
    variants = {0: 'grid-stride', 4: 'blocked', 12: 'blocked+nontemporal'}   # MEP_PROBE_BLOCKED / _NT
    for mode, key, factor in ((0, 'copy', 2), (1, 'read', 1), (2, 'write', 1)):
        best, how = 0.0, None
        for flags, vname in variants.items():
            for n_wg in (1024, 2048, 4096):
                def go():
                    _lib.call('mep_hbm_probe', ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), n16,
                              mode | flags, n_wg)
                go()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = 10
                a.record()
                for _ in range(reps):
                    go()
                b.record()
                torch.cuda.synchronize()
                rate = factor * 16 * n16 * reps / (a.elapsed_time(b) / 1e3) / 1e9
                if rate > best:
                    best, how = rate, '%s, %d workgroups' % (vname, n_wg)
        out[key + '_GBps'] = round(best, 1)
        out[key + '_best'] = how
    out.update(buffer_GiB=gib, kernel='mep_hbm_probe (csrc/probe.hip): dwordx4 streams, 8 loads in flight per '
               'thread; best of grid-stride / blocked / blocked nontemporal orders x 1024 / 2048 / 4096 workgroups',
               guide_GBps=6290.0,
               guide='MI355X_MICROARCH.md: 6.29 TB/s measured float4 copy (79% of the 8 TB/s spec)')
    del src, dst
    torch.cuda.empty_cache()
    return out


# launch name -> kernel symbol prefix (or prefixes) in the rocprofv3 summaries (scripts/parse_prof.py);
# mep_rfw_epi_* runs k_rfs_* on the large launches (State_Transfer) and k_rfw_* on the small ones
KERNEL_OF = {'mep_attn_bwd': 'k_attn_bwd', 'mep_attn_fwd': 'k_attn_fwd', 'mep_block_epi_fwd': 'k_epi_fwd',
             'mep_block_epi_bwd': 'k_epi_bwd', 'mep_wgrad': 'k_wgrad', 'mep_unify': 'k_unify',
             'mep_pool_fwd': 'k_pool_fwd', 'mep_pool_bwd': 'k_pool_bwd', 'mep_gemm': 'k_gemm', 'mep_tgemm': 'k_tgemm',
             'mep_rf_epi_fwd': 'k_rf_epi_fwd', 'mep_rf_epi_bwd': 'k_rf_epi_bwd', 'mep_sum_rows': 'k_sum_rows',
             'mep_wgemm': 'k_wgemm', 'mep_wgemm_ws': 'k_wgemm_ws', 'mep_wgemm_sum': 'k_wgemm_sum',
             'mep_rfw_front': 'k_rfw_front', 'mep_rfw_epi_fwd': ('k_rfs_fwd', 'k_rfw_fwd'),
             'mep_rfw_epi_bwd': ('k_rfs_bwd', 'k_rfw_bwd'),
             'mep_wsplit': 'k_wsplit', 'mep_reduce_grads': 'k_reduce_grads', 'mep_head_fwd_bwd': 'k_head',
             'mep_clip_adam_ext': 'k_clip_adam', 'mep_rf_head': 'k_rf_head'}


def pmc_traffic(launch, tag='cfg3'):
    """(HBM bytes per dispatch, source file) of the kernel behind `launch` from the newest
    committed PMC pass of this workload that measured it (profiles/r<round>_v<n>_pmc.json for cfg3
    fp32, profiles/r<round>_v<n>_pmc_<config>[_bf16].json for the others), or (None, None).
    Round 4 on (scripts/r4_traffic.py): reads = 32 x TCC_EA0_RDREQ_{DRAM,GMI,IO}_32B_sum, exact for
    every request size, writes = 1024 x WRITE_SIZE.  Rounds 2-3 used (2 FETCH_SIZE + WRITE_SIZE) x
    1024, which the r04 calibration (profiles/r04_fetch_cal.json) shows exact only for whole-line
    (128-B) reads -- FETCH_SIZE counts 64-B requests (half-line reads such as the attention's 64-byte
    head slices) at their full size, so the x2 doubled those."""
    def key(f):
        return [int(x) for x in re.findall(r'\d+', os.path.basename(f))]
    prefix = KERNEL_OF.get(launch)
    if prefix is None:
        return None, None
    pat = 'r*_v*_pmc.json' if tag == 'cfg3' else 'r*_v*_pmc_%s.json' % tag
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', pat)), key=key, reverse=True):
        for k, v in json.load(open(f)).items():
            if launch == 'mep_wgemm' and k.startswith(('k_wgemm_ws', 'k_wgemm_sum')):
                continue                                 # the prefix of the other GEMM
            if k.startswith(prefix) and isinstance(v, dict) and 'hbm_bytes_per_dispatch' in v:
                return int(v['hbm_bytes_per_dispatch']), os.path.relpath(f, ROOT)
    return None, None


def pmc_valu(launch, tag='cfg3'):
    """(VALU instructions per dispatch, source file) of the kernels behind `launch` from the newest
    committed SQ counter pass of this workload (profiles/r<round>_counters_<tag>.json, SQ_INSTS_VALU),
    or (None, None)."""
    prefix = KERNEL_OF.get(launch)
    if prefix is None:
        return None, None
    flat = {q for p in KERNEL_OF.values() for q in (p if isinstance(p, tuple) else (p,))}
    mine = prefix if isinstance(prefix, tuple) else (prefix,)
    longer = tuple(p for p in flat if p not in mine and p.startswith(mine))
    files = glob.glob(os.path.join(ROOT, 'profiles', 'r*_counters_%s.json' % tag))
    for f in sorted(files, key=lambda f: [int(x) for x in re.findall(r'\d+', os.path.basename(f))], reverse=True):
        tot = 0.0
        for k, v in json.load(open(f)).items():
            if k.startswith(prefix) and not (longer and k.startswith(longer)) and isinstance(v, dict):
                tot += float(v.get('raw', {}).get('SQ_INSTS_VALU', 0.0))
        if tot > 0:
            return tot, os.path.relpath(f, ROOT)
    return None, None


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


def host_cpus():
    """(CPUs this process may run on, the cgroup CPU quota or None): a GPU box's affinity mask can
    list the whole machine while its cgroup grants a share of it"""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return aff, quota


def timed_cpu(step, budget_s, max_steps=200):
    step()                                   # warmup
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if (n >= 3 and el >= budget_s) or n >= max_steps:
            return n, el


# ------------------------------------------------------------------------------ workloads
class Cfg3:
    """cmu-mosei Concat_Trans training step (BASELINE cfg3 / cfg4)."""
    name = 'cfg3'
    metric = METRIC
    unit = 'utt/s'
    baseline_dtype = 'bf16'       # BASELINE.json configs[2]: "Full tri-modal fusion ... bf16"

    def __init__(self, dev, rank, graph, bf16=False):
        from mep_amd import cmu_mosei
        from mep_amd.engine import TrainEngine
        from mep_amd.optim import FusedAdamW
        torch.manual_seed(0)
        self.bf16 = bf16
        self.model = cmu_mosei.Concat_Trans(dim=D, l_len=T, v_len=T, a_len=T, n_heads=H, n_layers=NL,
                                            ffn=1).to(dev).train()
        self.model.mep_precision = "bf16" if bf16 else "fp32"   # = running under autocast(bfloat16)
        self.opt = FusedAdamW(self.model, lr=1e-3)
        self.eng = TrainEngine(self.model, self.opt, clip=1.0, graph=graph)
        self.eng_eager = TrainEngine(self.model, self.opt, clip=1.0, graph=False)
        rng = np.random.default_rng(20261015 + rank)
        f = lambda d: torch.from_numpy(rng.standard_normal((B, 2, T, d), dtype=np.float32)).to(dev)  # noqa: E731
        l, v, a = (f(d) for d in DIMS)
        m = torch.ones(B, 2, T, device=dev)
        labels = torch.from_numpy((rng.random((B, 7)) < 0.3).astype(np.int64)).to(dev)
        self.plan = self.model.mep_runner(dev).plan(B, (T, T, T))
        self.plan.set_inputs(l, v, a, m, m.clone(), m.clone(), labels)
        self.rows = B

    def step(self):
        self.eng.step_plan(self.plan)

    def eager_step(self):
        self.eng_eager.step_plan(self.plan)

    def step_body(self):
        """the body the engine captures for one step: forward, backward, clip + AdamW"""
        self.eng._fwd_bwd_allreduce(self.plan, self.eng._runner(self.plan.device))
        self.eng._opt()

    def loss(self):
        return float(self.plan.loss.item())

    def config(self, world, graph):
        return {'workload': 'cmu-mosei Concat_Trans train step (fwd+bwd+clip+AdamW), BASELINE cfg3/cfg4',
                'global_batch': B * world, 'per_gpu_batch': B, 'seq_len': T, 'dims': list(DIMS), 'D': D,
                'heads': H, 'n_layers': NL, 'parallelism': 'dp%d' % world, 'graph': graph}

    @staticmethod
    def cpu_baseline(budget_s):
        """The CPU oracle (repo restatement of the reference path, fp32 PyTorch CPU): fwd+bwd+clip+
        AdamW at B=64, T=50."""
        from oracle import cmu_mosei as ocmu
        from oracle import common
        from tests.golden import specs
        from mep_amd import cmu_mosei
        m = cmu_mosei.Concat_Trans(dim=D, l_len=T, v_len=T, a_len=T, n_heads=H, n_layers=NL, ffn=1)
        shapes = {k: list(v.shape) for k, v in m.state_dict().items()}
        P = {k: torch.tensor(v, requires_grad=True) for k, v in specs.param_values(shapes, 1).items()}
        opt = common.AdamState(P.values(), lr=1e-3, weight_decay=0.01)
        batch = [torch.from_numpy(x) for x in specs.cmu_batch(seed=5, B=B, T=T, no_name_rows=(), full_masks=True)]
        n, el = timed_cpu(lambda: ocmu.train_step(P, opt, batch, H, NL), budget_s)
        return dict(value=round(B * n / el, 2), unit='utt/s', n=n, rows=B,
                    sample='%d steps of B=64,T=50 Concat_Trans fwd+bwd+clip+AdamW (oracle, fp32 CPU)' % n)


class Cfg5:
    """Ren-MME Base_model training step at T=300 (BASELINE cfg5): 32 rows = 16 duplicate pairs per
    GPU, text / video / audio d = 768 / 640 / 205, D=128, H=8, DROP=0.1, circle loss + R-Drop KL,
    AdamW."""
    name = 'cfg5'
    metric = 'rows/sec fwd+bwd, Ren-MME Base_model T=300 (d=768/640/205), 32 rows per MI355X'
    unit = 'rows/s'
    baseline_dtype = 'bf16'       # BASELINE.json configs[4]: "Ren-MME long-sequence config ... bf16"
    R, TT, DIMS5 = 32, 300, (768, 640, 205)

    def __init__(self, dev, rank, graph, bf16=False):
        from mep_amd import ren_mme
        from mep_amd.engine import TrainEngine
        from mep_amd.optim import FusedAdamW
        torch.manual_seed(0)
        R, TT = self.R, self.TT
        self.bf16 = bf16
        self.model = ren_mme.Base_model(dim=128, l_len=TT, v_len=TT, a_len=TT, n_heads=8, n_layers=1,
                                        ffn=1).to(dev).train()
        self.model.mep_precision = "bf16" if bf16 else "fp32"
        self.opt = FusedAdamW(self.model, lr=1e-3)
        self.eng = TrainEngine(self.model, self.opt, clip=1.0, rdrop=True, graph=graph)
        self.eng_eager = TrainEngine(self.model, self.opt, clip=1.0, rdrop=True, graph=False)
        rng = np.random.default_rng(20261015 + rank)
        feats = []
        for d in self.DIMS5:            # (prev, cur) per modality, every sample twice (R-Drop)
            pair = []
            for _ in range(2):
                x = rng.standard_normal((R // 2, TT, d), dtype=np.float32)
                pair.append(torch.from_numpy(np.repeat(x, 2, 0)).to(dev))
            feats.append(tuple(pair))
        m = torch.ones(R, TT, device=dev)
        labels = torch.from_numpy(np.repeat((rng.random((R // 2, 9)) < 0.3).astype(np.float32), 2, 0)).to(dev)
        runner = self.model.mep_runner(dev)
        self.plan = runner.plan(R, (TT, TT, TT))
        self.plan.set_inputs(*feats, (m, m), (m, m), (m, m), labels)
        self.rows = R

    def step(self):
        self.eng.step_plan(self.plan)

    def eager_step(self):
        self.eng_eager.step_plan(self.plan)

    def step_body(self):
        """the body the engine captures for one step: forward, backward, clip + AdamW"""
        self.eng._fwd_bwd_allreduce(self.plan, self.eng._runner(self.plan.device))
        self.eng._opt()

    def loss(self):
        return float(self.plan.loss.item())

    def config(self, world, graph):
        return {'workload': 'Ren-MME Base_model train step (fwd+bwd+R-Drop KL+clip+AdamW), BASELINE cfg5',
                'global_batch': self.R * world, 'per_gpu_batch': self.R, 'seq_len': self.TT,
                'dims': list(self.DIMS5), 'D': 128, 'heads': 8, 'n_layers': 1, 'dropout': 0.1,
                'parallelism': 'dp%d' % world, 'graph': graph}

    @classmethod
    def cpu_baseline(cls, budget_s):
        """The CPU oracle's Ren-MME step (fp32 CPU) on the same shape."""
        from oracle import common
        from oracle import ren_mme as oren
        from tests.golden import specs
        from mep_amd import ren_mme
        m = ren_mme.Base_model(dim=128, l_len=cls.TT, v_len=cls.TT, a_len=cls.TT, n_heads=8, n_layers=1, ffn=1)
        shapes = {k: list(v.shape) for k, v in m.state_dict().items()}
        P = {k: torch.tensor(v, requires_grad=True) for k, v in specs.param_values(shapes, 1).items()}
        opt = common.AdamState(P.values(), lr=1e-3, weight_decay=0.01)
        inputs, labels = specs.ren_batch(seed=5, pairs=cls.R // 2, T=cls.TT)
        inputs = [torch.from_numpy(x) for x in inputs]
        labels = torch.from_numpy(labels)
        drop = torch.nn.Dropout(0.1).train()      # DROP = 0.1 at both sites of every block, as the GPU step
        n, el = timed_cpu(lambda: oren.train_step(P, opt, inputs, labels, 8, 1, dropout=drop), budget_s, max_steps=50)
        return dict(value=round(cls.R * n / el, 3), unit='rows/s', n=n, rows=cls.R,
                    sample='%d steps of 32 rows (16 pairs), T=300, Ren-MME Base_model fwd+bwd+KL+clip+AdamW '
                           '(oracle, fp32 CPU, DROP 0.1)' % n)


class Cfg2:
    """realformer text encoder (BASELINE cfg2): Conv1d unify + position embedding + the first two
    residual blocks of the linguistic chain (others/realformer.py:224-233), B=64, T=50, d=300,
    D=96, H=6, FFN 2; backward of mean(out * G) (G fixed, seeded) + Adam (lr 1e-3)."""
    name = 'cfg2'
    metric = 'rows/sec fwd+bwd, realformer text encoder (2 residual blocks) B=64 T=50 d=300'
    unit = 'rows/s'
    baseline_dtype = 'fp32'       # BASELINE.json configs[1]: "... realformer attention only) fp32"

    def __init__(self, dev, rank, graph, bf16=False):
        from mep_amd import realformer as rf
        assert not bf16, 'cfg2 (realformer text encoder) is an fp32 configuration (BASELINE.json)'
        self.bf16 = False
        torch.manual_seed(0)
        self.mc = rf.Multi_class(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=T, v_len=T, a_len=T, n_heads=6,
                                 n_layers=2, ffn=2).to(dev).train()
        self.runner = runner = self.mc.mep_chain_runner(2, dev)
        rng = np.random.default_rng(20261015 + rank)
        x = torch.from_numpy(rng.standard_normal((B, T, 300), dtype=np.float32)).to(dev)
        m = torch.ones(B, T, device=dev)
        G = torch.from_numpy(rng.standard_normal((B, T, 96), dtype=np.float32)).to(dev)
        self.plan = runner.plan(B, 1)
        z = torch.zeros(0, device=dev)
        self.plan.set_inputs(x, z, z, m, z, z)
        self.G = G.reshape(self.plan.dout_chain.shape)
        self.plan.dout_chain.copy_(self.G / G.numel())   # d mean(out * G) / d out
        self.opt = _FlatAdam(runner.flat, lr=1e-3)
        if os.environ.get('MEP_NORM_FOLD', '1') != '0':
            self.opt.fold_into(self.plan)
        self.graph = graph
        self.g = None
        self.rows = B

    def _body(self):
        self.plan.forward(grad=True)
        self.plan.backward()
        self.opt.step()

    def step(self):
        if not self.graph:
            self._body()
            return
        if self.g is None:
            self._body()
            torch.cuda.synchronize()
            self.g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g):
                self._body()
        self.g.replay()

    def eager_step(self):
        self._body()

    def step_body(self):
        self._body()

    def loss(self):
        """The objective mean(out * G) of the last step's forward."""
        return float((self.plan.out_chain * self.G).double().mean().item())

    def config(self, world, graph):
        return {'workload': 'realformer text encoder fwd+bwd+Adam (Conv1d unify + pos + 2 residual blocks), '
                            'BASELINE cfg2', 'global_batch': B * world, 'per_gpu_batch': B, 'seq_len': T,
                'dims': [300], 'D': 96, 'heads': 6, 'n_layers': 2, 'ffn': 2, 'parallelism': 'dp%d' % world,
                'graph': graph}

    @staticmethod
    def cpu_baseline(budget_s):
        """The CPU oracle's realformer chain fwd+bwd + torch Adam (fp32 CPU) on the same shape."""
        from oracle import common
        from oracle import realformer as orf
        from tests.golden import specs
        from mep_amd import realformer as rf
        mc = rf.Multi_class(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=T, v_len=T, a_len=T, n_heads=6,
                            n_layers=2, ffn=2)
        shapes = {k: list(v.shape) for k, v in mc.state_dict().items()}
        P = {k: torch.tensor(v, requires_grad=True) for k, v in specs.param_values(shapes, 1).items()}
        used = [k for k in P if k.startswith(('unify_dimension.linguistic', 'linguistic_position',
                                             'multimodal_blocks.0.', 'multimodal_blocks.1.'))]
        opt = torch.optim.Adam([P[k] for k in used], lr=1e-3)
        rng = np.random.default_rng(5)
        x = torch.from_numpy(rng.standard_normal((B, T, 300), dtype=np.float32))
        lm = torch.ones(B, T)
        G = torch.from_numpy(rng.standard_normal((B, T, 96), dtype=np.float32))

        def step():
            opt.zero_grad()
            w = P['unify_dimension.linguistic.weight'][:, :, 0]
            h0 = common.linear(x, w) + P['linguistic_position.position_embeddings.weight'][:T].unsqueeze(0)
            h, _ = orf.encode_chain(P, '', h0, 2, 6, lm)
            (h * G).mean().backward()
            opt.step()
        n, el = timed_cpu(step, budget_s)
        return dict(value=round(B * n / el, 2), unit='rows/s', n=n, rows=B,
                    sample='%d steps of B=64,T=50 realformer text chain fwd+bwd+Adam (oracle, fp32 CPU)' % n)


class RfState:
    """realformer State_Transfer training step at the reference's own configuration
    (others/realformer.py:23-38: BATCH 64, P_LEN 6 utterances, L/V/A_LEN 50, DIM 96, N_HEADS 6,
    N_LAYERS 2, FFN 2): the shared Multi_class encoder over all B x P utterances, the
    State_Transfer head with its gate recurrence over the 6 utterances (:266-286), the masked
    circle loss (:311-312), clip_grad_norm_(1.0) and Adam (lr 1e-3, no weight decay; :342).  One
    row = one sequence of 6 utterances.  Synthetic N(0,1) features, all-ones frame and utterance
    masks, Bernoulli(0.3) labels.  fp32 (the reference has no AMP)."""
    name = 'rfstate'
    metric = 'sequences/sec fwd+bwd, realformer State_Transfer B=64 P=6 T=50 (d=300/35/74)'
    unit = 'seq/s'
    baseline_dtype = 'fp32'
    P = 6

    def __init__(self, dev, rank, graph, bf16=False):
        from mep_amd import realformer as rf
        from mep_amd.engine import TrainEngine
        from mep_amd.optim import FusedAdam
        assert not bf16, 'rfstate is an fp32 workload (the reference has no AMP)'
        self.bf16 = False
        torch.manual_seed(0)
        self.model = rf.State_Transfer(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=T, v_len=T, a_len=T, n_heads=6,
                                       n_layers=2, ffn=2).to(dev).train()
        self.opt = FusedAdam(self.model, lr=1e-3)
        self.eng = TrainEngine(self.model, self.opt, clip=1.0, graph=graph)
        self.eng_eager = TrainEngine(self.model, self.opt, clip=1.0, graph=False)
        rng = np.random.default_rng(20261015 + rank)
        f = lambda d: torch.from_numpy(rng.standard_normal((B, self.P, T, d), dtype=np.float32)).to(dev)  # noqa: E731
        l, v, a = (f(d) for d in DIMS)
        m = torch.ones(B, self.P, T, device=dev)
        labels = torch.from_numpy((rng.random((B, self.P, 6)) < 0.3).astype(np.int64)).to(dev)
        um = torch.ones(B, self.P, dtype=torch.int64, device=dev)
        self.plan = self.model.mep_runner(dev).stage(l, v, a, labels, m, m.clone(), m.clone(), um)
        self.rows = B

    def step(self):
        self.eng.step_plan(self.plan)

    def eager_step(self):
        self.eng_eager.step_plan(self.plan)

    def step_body(self):
        self.eng._fwd_bwd_allreduce(self.plan, self.eng._runner(self.plan.device))
        self.eng._opt()

    def loss(self):
        return float(self.plan.loss.item())

    def config(self, world, graph):
        return {'workload': 'realformer State_Transfer train step (fwd+bwd+clip+Adam), reference configuration',
                'global_batch': B * world, 'per_gpu_batch': B, 'utterances_per_row': self.P, 'seq_len': T,
                'dims': list(DIMS), 'D': 96, 'heads': 6, 'n_layers': 2, 'ffn': 2, 'parallelism': 'dp%d' % world,
                'graph': graph}

    @classmethod
    def cpu_baseline(cls, budget_s):
        """The CPU oracle's State_Transfer step (fp32 CPU, Adam) on the same shape."""
        from oracle import common
        from oracle import realformer as orf
        from tests.golden import specs
        from mep_amd import realformer as rf
        m = rf.State_Transfer(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=T, v_len=T, a_len=T, n_heads=6,
                              n_layers=2, ffn=2)
        shapes = {k: list(v.shape) for k, v in m.state_dict().items()}
        P = {k: torch.tensor(v, requires_grad=True) for k, v in specs.param_values(shapes, 1).items()}
        opt = common.AdamState(P.values(), lr=1e-3, weight_decay=0.0, decoupled=False)
        batch = [torch.from_numpy(x) for x in specs.realformer_batch(seed=5, B=B, P=cls.P, T=T)]
        n, el = timed_cpu(lambda: orf.train_step(P, opt, batch, 6, 2), budget_s, max_steps=50)
        return dict(value=round(B * n / el, 3), unit='seq/s', n=n, rows=B,
                    sample='%d steps of B=64 sequences x 6 utterances, T=50, State_Transfer fwd+bwd+clip+Adam '
                           '(oracle, fp32 CPU)' % n)


class _FlatAdam:
    """Adam (weight decay 0, no clip: others/realformer.py:342) over a runner's flat buffer with the
    fused clip+Adam kernel (mep_clip_adam), graph-capturable."""

    def __init__(self, flat, lr):
        import ctypes
        from mep_amd import _lib
        self.flat, self._lib, self.ct = flat, _lib, ctypes
        dev = flat.buf.device
        self.exp_avg = torch.zeros_like(flat.buf)
        self.exp_avg_sq = torch.zeros_like(flat.buf)
        # workspace: [0, 1024) the norm pass's partials and the step scalars, then the partials of a
        # backward reduction that folded the norm pass in (optim.py MAX_EXT)
        self.partial = torch.zeros(1024 + (1 << 16), dtype=torch.float32, device=dev)
        self.n_ext = 0
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.hyper = torch.tensor([lr, 0.9, 0.999, 1e-8, 0.0, float('inf'), 1.0, 0.0], dtype=torch.float32,
                                  device=dev)

    def fold_into(self, plan):
        """the norm pass (and the step counter) folded into the plan's backward reduction"""
        plan.norm_fold = (self.partial.data_ptr(), self.step_t.data_ptr(), self.hyper.data_ptr())
        self.n_ext = plan.reduce_grid()
        assert 0 < self.n_ext <= 1 << 16

    def step(self):
        P = self.ct.c_void_p
        segs = (self._lib.Seg * 1)(self._lib.Seg(0, self.flat.n_grad))
        self._lib.call('mep_clip_adam_ext', P(self.flat.buf.data_ptr()), P(self.flat.grad.data_ptr()),
                       P(self.exp_avg.data_ptr()), P(self.exp_avg_sq.data_ptr()), self.ct.cast(segs, P), 1,
                       self.flat.total, P(self.partial.data_ptr()), P(self.gnorm.data_ptr()),
                       P(self.hyper.data_ptr()), P(self.step_t.data_ptr()), 0, self.n_ext)


CONFIGS = {'cfg3': Cfg3, 'cfg5': Cfg5, 'cfg2': Cfg2, 'rfstate': RfState}


def roofline_of(work, name, tot, costs, probe=None):
    """roofline object of launch `name`: the plan's algorithmic flops / bytes per launch over the
    launch's in-step time (time_launches), plus the committed PMC traffic and, when
    measured, the fraction of the box's measured HBM peak"""
    from mep_amd import roofline
    t, n = tot[name]
    per_launch_s = t / n
    flops, nbytes = costs[name]
    spec = getattr(work.plan, 'spec', None)
    tag = work.name + ('_bf16' if work.bf16 else '')
    valu, vsrc = pmc_valu(name, tag)
    rl = roofline.roofline_entry(name, flops / n, nbytes / n, per_launch_s, bf16=work.bf16, D=getattr(spec, 'D', None),
                                 valu=(valu / n, vsrc) if valu else None)
    rl['traffic'], rl['traffic_source'] = pmc_traffic(name, tag)
    rl['avg_launch_us'] = round(per_launch_s * 1e6, 2)
    rl['launches_per_step'] = n
    if probe and rl['bound'] == 'hbm':
        rl['peak_measured'] = probe['read_GBps']
        rl['frac_measured'] = round(rl['achieved'] / probe['read_GBps'], 4)
        rl['frac_guide'] = round(rl['achieved'] / probe['guide_GBps'], 4)
    return rl


def roofline_all(work, tot, costs, probe=None):
    """every priced launch of the step: {launch: roofline object} (bound, frac, VALU floor, limiter)"""
    return {k: roofline_of(work, k, tot, costs, probe) for k in sorted(tot, key=lambda k: -tot[k][0]) if k in costs}


def run_config(cls, dev, rank, world, graph, bf16, steps, warmup):
    """time `steps` steps of one workload at one precision, then its launches one by one"""
    from mep_amd import _lib, roofline
    work = cls(dev, rank, graph, bf16=bf16)
    for _ in range(warmup):
        work.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        work.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    loss = work.loss()

    # every launch of the step, timed where it runs (time_launches)
    tot, method = time_launches(work)
    costs = roofline.launch_costs(work.plan)
    kernels = {k: dict(ms_per_step=round(t * 1e3, 4), launches_per_step=n, avg_launch_us=round(t / n * 1e6, 2))
               for k, (t, n) in sorted(tot.items(), key=lambda kv: -kv[1][0])}
    dom = max((k for k in tot if k in costs), key=lambda k: tot[k][0])
    res = {
        'value': round(work.rows * world * steps / el, 2),
        'ms_per_step': round(el / steps * 1e3, 4),
        'loss': round(loss, 6),
        'kernels': kernels,
        'kernels_sum_ms': round(sum(t for t, _ in tot.values()) * 1e3, 4),
        'kernel_timing': method,
    }
    return work, res, tot, costs, dom


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, selftest=False):
    """`bench.py --gpus N` started without WORLD_SIZE: run N fresh child ranks, one per GPU, under
    torch.distributed.run (127.0.0.1 rendezvous) and exit with its code.  The children inherit
    stdout, so rank 0's JSON line is the only line printed.  This parent makes no HIP call and does
    not exec: torch.cuda.device_count() does not initialise the GPU on this image."""
    import subprocess
    if not selftest:
        have = torch.cuda.device_count()
        if have < n:
            print('bench.py: --gpus %d needs %d GPUs, this node has %d; refusing to report a %d-GPU line'
                  % (n, n, have, n), file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=%d' % n,
           '--master-addr=127.0.0.1', '--master-port=%d' % free_port(), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')     # dmabuf IPC (RCCL / shared CUDA tensors)
    return subprocess.call(cmd, env=env)


def rank_devices(dev, world):
    """[(rank, local rank, device index, PCI bus id)] of every rank (rank 0 reports them all)"""
    p = torch.cuda.get_device_properties(dev)
    mine = [int(os.environ.get('RANK', '0')), int(os.environ.get('LOCAL_RANK', '0')), dev.index,
            '%04x:%02x:%02x' % (getattr(p, 'pci_domain_id', 0), getattr(p, 'pci_bus_id', 0),
                                getattr(p, 'pci_device_id', 0))]
    if world == 1:
        return [mine]
    got = [None] * world
    dist.all_gather_object(got, mine)
    return got


def launch_selftest(world, rank):
    """--launch-selftest (CPU tests): the ranks started by launch_ranks join a gloo group, SUM
    their rank ids and rank 0 prints one line -- the launcher path without a GPU."""
    if world > 1:
        dist.init_process_group('gloo')
    t = torch.tensor([float(rank + 1)])
    if world > 1:
        dist.all_reduce(t)
    ranks = [rank]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, rank)
    if rank == 0:
        print(json.dumps({'metric': 'launcher self-test', 'n_gpus': world, 'rccl_world': world,
                          'ranks': ranks, 'rank_sum': float(t.item()), 'pid': os.getpid()}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--launch-selftest', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', default='cfg3', choices=sorted(CONFIGS))
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--no-bf16', action='store_true', help='skip the nested bf16 line of cfg3 / cfg5')
    ap.add_argument('--no-probe', action='store_true', help='skip the measured HBM peak')
    ap.add_argument('--cpu-budget', type=float, default=12.0)
    ap.add_argument('--dtype', default='fp32', choices=('fp32', 'bf16'),
                    help="fp32 (default): the reference's own precision, the 1e-4 parity path; the "
                         "config's BASELINE bf16 line is nested in the same JSON")
    args = ap.parse_args()
    cls = CONFIGS[args.config]
    if args.gpus < 1:
        ap.error('--gpus must be >= 1')

    env_world = os.environ.get('WORLD_SIZE')
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:], selftest=args.launch_selftest)
    world = int(env_world or '1')
    if world != args.gpus:
        print('bench.py: --gpus %d but WORLD_SIZE=%d; launch one rank per GPU with matching counts'
              % (args.gpus, world), file=sys.stderr, flush=True)
        return 2
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.launch_selftest:
        return launch_selftest(world, rank)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    devices = rank_devices(dev, world)
    rccl_world = dist.get_world_size() if world > 1 else 1
    if world > 1 and len({d[3] for d in devices}) != world:
        print('bench.py: ranks share a GPU: %s' % devices, file=sys.stderr, flush=True)
        return 2

    from mep_amd import _lib
    graph = not args.no_graph
    probe = None if args.no_probe else hbm_probe(dev)
    work, res, tot, costs, dom = run_config(cls, dev, rank, world, graph, args.dtype == 'bf16', args.steps,
                                            args.warmup)
    out = {
        'metric': work.metric,
        'value': res['value'],
        'unit': work.unit,
        'n_gpus': world,
        'rccl_world': rccl_world,
        'rank_devices': devices,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': res['ms_per_step'],
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': args.dtype,
        'data': 'synthetic N(0,1) features, all-ones masks, Bernoulli(0.3) labels, random-init weights',
        'config': work.config(world, graph),
        'loss': res['loss'],
        'roofline': roofline_of(work, dom, tot, costs, probe),
        'roofline_attention': roofline_of(work, 'mep_attn_bwd', tot, costs, probe),
        'rooflines': roofline_all(work, tot, costs, probe),
        'kernels': res['kernels'],
        'kernels_sum_ms': res['kernels_sum_ms'],
        'kernel_timing': res['kernel_timing'],
    }
    if probe:
        out['hbm_measured'] = probe
    del work
    torch.cuda.empty_cache()
    if args.dtype == 'fp32' and cls.baseline_dtype == 'bf16' and not args.no_bf16:
        # BASELINE.json names bf16 for this config: the bf16 path's line, same steps, same box
        w2, r2, tot2, costs2, dom2 = run_config(cls, dev, rank, world, graph, True, args.steps, args.warmup)
        r2['roofline'] = roofline_of(w2, dom2, tot2, costs2, probe)
        r2['roofline_attention'] = roofline_of(w2, 'mep_attn_bwd', tot2, costs2, probe)
        r2['rooflines'] = roofline_all(w2, tot2, costs2, probe)
        r2['dtype'] = 'bf16'
        out['bf16'] = r2
        del w2
        torch.cuda.empty_cache()
    out['switches'] = {'read': {k: v['value'] for k, v in sorted(_lib.SWITCHES.items())},
                       'set_in_env': _lib.switches_from_env()}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the oracle on the box's host cores -- every CPU this process may use
        # (capped by the cgroup quota when there is one)
        aff, quota = host_cpus()
        threads = min(aff, quota) if quota else aff
        torch.set_num_threads(threads)
        cb = cls.cpu_baseline(args.cpu_budget)
        cb.update(cores=torch.get_num_threads(), kind='port', cpu_model=cpu_model(), affinity_cpus=aff,
                  cgroup_cpus=quota)
        out['cpu_baseline'] = cb
        out['gpu_vs_cpu'] = round(out['value'] / cb['value'], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
