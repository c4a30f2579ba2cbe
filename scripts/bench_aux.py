"""Measurement of the SURVEY 8(f) rows next to the hot path: device-side batch assembly
(mep_assemble_windows) and the evaluation threshold sweep (mep_threshold_sweep), each beside the
reference's CPU formulation (the oracle restatement, single-threaded numpy / sklearn).

Prints one JSON line per row.  Synthetic CMU-MOSEI-shaped data: 2,000 utterances, text
L ~ U{5..60} x 300, visual L ~ U{20..400} x 35, audio L ~ U{50..1500} x 74 (fp32; ~100 Hz COVAREP),
B = 64 pairs per batch, L_LEN = V_LEN = A_LEN = 50 (BASELINE cfg3).
Usage: python scripts/bench_aux.py [--iters 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()
from mep_amd import _lib, batching, evaluate  # noqa: E402
from oracle import batching as ob  # noqa: E402  (CPU baseline leg only)
from oracle import evaluate as oev  # noqa: E402

HBM_PEAK = 8000.0


class StreamTimer:
    """HIP events recorded on the launching stream around every named launch (as bench.py)."""

    def __init__(self):
        self.ev = {}

    def begin(self, name, stream):
        s = stream or torch.cuda.current_stream()
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        self.ev.setdefault(name, []).append([e, None])

    def end(self, name, stream):
        s = stream or torch.cuda.current_stream()
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        self.ev[name][-1][1] = e

    def mean_ms(self, name):
        torch.cuda.synchronize()
        v = [a.elapsed_time(b) for a, b in self.ev.get(name, [])]
        return float(np.mean(v)) if v else None


def make_data(rng, n=2000):
    a_max = int(os.environ.get('AUX_AUDIO_MAX', '1500'))   # longest audio sequence (frames)
    spec = {'linguistic': (5, 60, 300), 'visual': (20, 400, 35), 'acoustic': (50, a_max, 74)}
    data = {m: {} for m in spec}
    for i in range(n):
        for m, (lo, hi, d) in spec.items():
            L = int(rng.integers(lo, hi + 1))
            x = rng.standard_normal((L, d)).astype(np.float32)
            if m == 'acoustic':
                x[rng.random(x.shape) < 1e-3] = -np.inf
            data[m]['u%d' % i] = x
    labels = {k: rng.integers(0, 2, 7) for k in data['linguistic']}
    return data, labels


def assembly_bytes(store, pairs, lens):
    """Algorithmic HBM bytes of one cmu batch: window frames + whole sequences for the summary rows
    read once, every slot + mask written once (4-byte elements)."""
    rd = wr = 0
    mods = batching.MODALITIES
    for prev, cur in pairs:
        two = store.length('linguistic', cur) >= lens[0] - 3
        for _ in ([1, 0] if two else [0]):
            for m, n in zip(mods, lens):
                d = store.dim(m)
                wr += 2 * (n * d + n) * 4
                for name in (prev, cur):
                    if name != batching.NO_NAME:
                        L = store.length(m, name)
                        rd += (min(L, n - 3) + L) * d * 4
    return rd + wr


def bench_assembly(args, rng):
    data, labels = make_data(rng)
    names = list(data['linguistic'])
    lens = (50, 50, 50)
    store = batching.FeatureStore(data, 'cuda')
    batches = []
    for b in range(args.iters + 5):
        idx = rng.integers(1, len(names), 64)
        batches.append([(names[i - 1] if i % 9 else batching.NO_NAME, names[i]) for i in idx])
    for p in batches[:5]:
        batching.cmu_batch(store, p, labels, lens)
    torch.cuda.synchronize()
    timer = StreamTimer()
    _lib.TIMER = timer
    t0 = time.perf_counter()
    rows = 0
    for p in batches[5:]:
        out = batching.cmu_batch(store, p, labels, lens)
        rows += out[-1].shape[0]
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    _lib.TIMER = None
    k_ms = timer.mean_ms('mep_assemble_windows')
    byts = np.mean([assembly_bytes(store, p, lens) for p in batches[5:10]])
    # CPU: the reference's numpy windowing for the same pairs (oracle restatement), 1 thread
    t0 = time.perf_counter()
    n_cpu, cpu_rows = 0, 0
    while time.perf_counter() - t0 < args.cpu_seconds and n_cpu < len(batches) - 5:
        out = ob.cmu_batch(data, labels, batches[5 + n_cpu], lens)
        cpu_rows += out[-1].shape[0]
        n_cpu += 1
    cpu_wall = time.perf_counter() - t0
    return {'metric': 'cmu batch assembly, batches/s (B=64 pairs, T=50)', 'row': 'SURVEY 8(f)1',
            'value': round(args.iters / wall, 1), 'unit': 'batches/s', 'rows_per_batch': rows / args.iters,
            'kernel': 'mep_assemble_windows', 'kernel_avg_us': round(k_ms * 1e3, 2),
            'roofline': {'bound': 'hbm', 'achieved': round(byts / (k_ms * 1e-3) / 1e9, 1), 'peak': HBM_PEAK,
                         'unit': 'GB/s', 'frac': round(byts / (k_ms * 1e-3) / 1e9 / HBM_PEAK, 4),
                         'algorithmic_bytes': int(byts)},
            'cpu_baseline': {'value': round(n_cpu / cpu_wall, 2), 'unit': 'batches/s', 'cores': 1, 'kind': 'port',
                             'sample': '%d batches of the same pairs, numpy masking()+data_loader restatement' % n_cpu}}


def bench_sweep(args, rng):
    N, C, n_thr = 4 * 1024 * 6, 6, 400        # ~4k test utterance lists x P_LEN = 6 rows
    p1 = torch.randn(N, C, device='cuda')
    p2 = torch.randn(N, C, device='cuda')
    lab = (torch.rand(N, C, device='cuda') < 0.3).long()
    thr = torch.from_numpy(evaluate.rf_thresholds(n_thr)).cuda()
    counts = torch.zeros(n_thr, C, 4, dtype=torch.int32, device='cuda')
    for _ in range(3):
        evaluate.threshold_sweep([p1, p2], lab, thr, weights=(0.6, 0.4), counts=counts)
    torch.cuda.synchronize()
    timer = StreamTimer()
    _lib.TIMER = timer
    t0 = time.perf_counter()
    for _ in range(args.iters):
        counts.zero_()
        evaluate.threshold_sweep([p1, p2], lab, thr, weights=(0.6, 0.4), counts=counts)
        evaluate.rf_select(counts, n_thr)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    _lib.TIMER = None
    k_ms = timer.mean_ms('mep_threshold_sweep')
    alg = N * C * (2 * 4 + 8) + n_thr * C * 4 * 4 * 2
    # CPU: the reference loop (list appends + sklearn per threshold) over the same scores; its
    # first threshold pass, x400, is a LOWER bound on the reference (its lists keep growing)
    pa, pb = p1.cpu().reshape(-1, 6, 6), p2.cpu().reshape(-1, 6, 6)
    lb = lab.cpu().reshape(-1, 6, 6)
    mk = torch.ones(pa.shape[0], 6, dtype=torch.long)
    t0 = time.perf_counter()
    oev.rf_test([(pa, pb, lb, mk)], 1)
    cpu_per_thr = time.perf_counter() - t0
    return {'metric': 'realformer ensemble threshold sweep (400 thresholds, 2 models), sweeps/s',
            'row': 'SURVEY 8(f)2', 'value': round(args.iters / wall, 1), 'unit': 'sweeps/s', 'rows': N,
            'kernel': 'mep_threshold_sweep', 'kernel_avg_us': round(k_ms * 1e3, 2),
            # sorted thresholds -> histogram path: per row C scores x 2 models (fp32) + C int64
            # labels read once, counts [n_thr, C, 4] int32 read+written once; latency-bound
            # (two launches, LDS/L2 atomics), far from the HBM roof at this size
            'roofline': {'bound': 'hbm', 'achieved': round(alg / (k_ms * 1e-3) / 1e9, 1), 'peak': HBM_PEAK,
                         'unit': 'GB/s', 'frac': round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK, 4),
                         'algorithmic_bytes': alg, 'path': 'sorted (histogram + suffix sums)'},
            'cpu_baseline': {'value': round(1.0 / (cpu_per_thr * n_thr), 5), 'unit': 'sweeps/s', 'cores': 1,
                             'kind': 'port', 'sample': 'first threshold pass of the reference loop over the same '
                                                       '%d rows (list appends + sklearn), x400' % N}}


def bench_train(args, rng):
    """cmu train() epochs (fused engine, B = 64 pairs, T = 50, D = 96) fed by the device loader vs
    by the reference-layout host loader (numpy windowing + zip/stack + H2D): utterance rows/s of
    the whole epoch, data loading included."""
    import random
    from mep_amd import cmu_mosei
    from mep_amd.optim import FusedAdamW
    data, labels = make_data(rng, n=1500)
    names = list(data['linguistic'])
    pairs = [(names[i - 1] if i % 9 else batching.NO_NAME, names[i]) for i in range(1, 1281)]  # 20 batches
    lens = (50, 50, 50)
    store = batching.FeatureStore(data, 'cuda')
    res = {}
    for kind in ('device', 'host'):
        torch.manual_seed(0)
        model = cmu_mosei.Concat_Trans(dim=96, l_len=50, v_len=50, a_len=50, n_heads=6, n_layers=1, ffn=1).cuda()
        opt = FusedAdamW(model, lr=1e-3)
        times = []
        for ep in range(3):                  # epoch 0 captures one graph per distinct row count
            random.seed(ep)
            order = list(pairs)
            if kind == 'device':
                it = batching.cmu_data_loader(store, lens)(order, labels, 64)
            else:
                random.shuffle(order)
                it = (list(zip(*ob.cmu_batch(data, labels, order[i:i + 64], lens))) for i in range(0, len(order), 64))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cmu_mosei.train(model, it, opt)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        res[kind] = min(times[1:])
    rows = sum(2 if store.length('linguistic', c) >= 47 else 1 for _, c in pairs)
    return {'metric': 'cmu train epoch incl. data loading, utterance rows/s (B=64 pairs, T=50)',
            'row': 'SURVEY 8(f)1 in the training loop', 'value': round(rows / res['device'], 1), 'unit': 'rows/s',
            'host_loader_value': round(rows / res['host'], 1), 'rows_per_epoch': rows, 'batches': 20,
            'note': 'host loader = numpy masking/data_loader restatement (1 core) + zip/stack + pinned H2D'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--only', default='')
    args = ap.parse_args()
    rng = np.random.default_rng(20261016)
    for name, fn in (('assembly', bench_assembly), ('sweep', bench_sweep), ('train', bench_train)):
        if args.only and args.only != name:
            continue
        print(json.dumps(fn(args, rng)), flush=True)


if __name__ == '__main__':
    main()
