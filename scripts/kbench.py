"""Per-kernel micro-benchmark of the bench workload's launches (for profiling one kernel at a time).

    python scripts/kbench.py [--kernel mep_attn_fwd] [--reps 50]
Builds the cfg3 plan (Concat_Trans D=96 H=6 B=64 T=50), runs one eager step, then replays the
chosen launch `reps` times and prints the average HIP-event time per launch.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kernel', default='all')
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--layers', type=int, default=1)
    ap.add_argument('--T', type=int, default=50)
    ap.add_argument('--config', default='cfg3', choices=('cfg3', 'cfg5'))
    ap.add_argument('--dtype', default='fp32', choices=('fp32', 'bf16'))
    args = ap.parse_args()
    import bench
    from mep_amd import _lib
    from mep_amd._lib import launch
    dev = torch.device('cuda:0')
    bench.T, bench.NL = args.T, args.layers
    work = bench.CONFIGS[args.config](dev, 0, graph=False, bf16=args.dtype == 'bf16')
    work.eager_step()
    torch.cuda.synchronize()
    p = work.plan
    D = p.spec.D
    pr = p.prec
    table = {
        'mep_unify': lambda: _lib.gemm('mep_unify', p.d_unify, p.t_unify, prec=pr),
        'mep_attn_fwd': lambda: launch('mep_attn_fwd', p.d_attn[0], p.t_attn[0], threads=p.g_attn[0][2] | pr),
        'mep_block_epi_fwd': lambda: launch('mep_block_epi_fwd', p.d_epi[0], p.t_epi[0], threads=D | pr),
        'mep_block_epi_bwd': lambda: launch('mep_block_epi_bwd', p.d_epib[0], p.t_epi[0], threads=D | pr),
        'mep_attn_bwd': lambda: launch('mep_attn_bwd', p.d_attnb[0], p.t_attnb[0], threads=p.f_attnb[0] | pr),
        'mep_wgrad': lambda: launch('mep_wgrad', p.d_wgrad, p.t_wgrad),
        'mep_pool_fwd': lambda: launch('mep_pool_fwd', p.d_pool, p.t_pool),
    }
    names = list(table) if args.kernel == 'all' else args.kernel.split(',')
    for name in names:
        fn = table[name]
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        print('%-20s %8.2f us/launch' % (name, a.elapsed_time(b) / args.reps * 1e3), flush=True)


if __name__ == '__main__':
    main()
