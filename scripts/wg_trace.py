"""Phase trace of the weight-gradient launch (development builds with -DMEP_WG_TRACE, csrc/gemm.hip):
    VARIANTS="trace=-DMEP_WG_TRACE" bash scripts/ab_build.sh
    MEP_LIB=variants/trace/lib.so python scripts/wg_trace.py [--dtype bf16] [--balance 0]
Runs the cfg3 bench plan's step eagerly, then the mep_wgrad launch alone, and prints over the
workgroups the spread of each phase's start (0 start, 1 main loop, 2 main loop end, 3 slot
written) relative to the earliest workgroup start, in microseconds (100 MHz real-time counter).
--balance 0: the uniform-chunk segments (MEP_WG_BALANCE=0) instead of trimodal.wgrad_counts."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dtype', default='fp32', choices=('fp32', 'bf16'))
    ap.add_argument('--balance', type=int, default=1)
    ap.add_argument('--reduce', type=int, default=0, help='1: trace the mep_reduce_grads launch instead')
    # (the trace build faulted on the State_Transfer workload, twice: traced on cfg3 only)
    ap.add_argument('--config', default='cfg3', choices=('cfg3',))
    args = ap.parse_args()
    import bench
    from mep_amd import _lib, trimodal
    from mep_amd._lib import launch
    trimodal.WG_BALANCE = bool(args.balance)
    dev = torch.device('cuda:0')
    kw = {} if args.config in ('cfg2', 'rfstate') else dict(bf16=args.dtype == 'bf16')
    work = bench.CONFIGS[args.config](dev, 0, graph=False, **kw)
    for _ in range(3):
        work.eager_step()
    torch.cuda.synchronize()
    p = work.plan
    if args.reduce:
        return trace_reduce(work, args)
    fn = _lib.lib().mep_wg_trace_read
    fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
    buf = np.zeros((8192, 8), dtype=np.uint64)
    for _ in range(3):
        launch('mep_wgrad', p.d_wgrad, p.t_wgrad)
        torch.cuda.synchronize()
        fn(buf.ctypes.data)
    nwg = p.t_wgrad
    t = buf[:nwg].astype(np.float64)
    t0 = t[:, 0][t[:, 0] > 0].min()
    us = np.where(t > 0, (t - t0) / 100.0, np.nan)
    print('%s, balance %d: %d workgroups, span %.2f us' % (args.dtype, args.balance, nwg, np.nanmax(us[:, 3])))
    for k, nm in enumerate(['start', 'loop', 'loop end', 'slot written']):
        q = np.nanpercentile(us[:, k], [0, 10, 50, 90, 100])
        print('  %-13s ' % nm + ' '.join('%7.2f' % v for v in q))


def trace_reduce(work, args):
    """k_reduce_grads blocks: start / job done / end per job kind, with the launch's norm pass on
    (the bench's engine plan folds the clip's norm into this launch)"""
    from mep_amd import _lib
    p = work.plan
    fn = _lib.lib().mep_rg_trace_read
    fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
    buf = np.zeros((8192, 4), dtype=np.int64)
    for _ in range(3):
        work.eager_step()
        torch.cuda.synchronize()
        fn(buf.ctypes.data)
    n = min(p.reduce_grid(), 8192)   # the trace buffer holds the first 8,192 blocks
    t = buf[:n].astype(np.float64)
    t0 = t[:, 0].min()
    us = (t[:, :3] - t0) / 100.0
    kind = buf[:n, 3]
    print('%s: %d blocks, span %.2f us' % (args.dtype, n, us[:, 2].max()))
    for k, nm in enumerate(['head', 'split sum', 'column sum', 'empty']):
        sel = kind == k
        if not sel.any():
            continue
        print('  %-10s %4d blocks  start %s  job %s  end %s' % (
            nm, int(sel.sum()), ' '.join('%6.2f' % v for v in np.percentile(us[sel, 0], [0, 50, 100])),
            ' '.join('%6.2f' % v for v in np.percentile(us[sel, 1] - us[sel, 0], [0, 50, 100])),
            ' '.join('%6.2f' % v for v in np.percentile(us[sel, 2], [0, 50, 100]))))


if __name__ == '__main__':
    main()
