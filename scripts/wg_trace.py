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
    args = ap.parse_args()
    import bench
    from mep_amd import _lib, trimodal
    from mep_amd._lib import launch
    trimodal.WG_BALANCE = bool(args.balance)
    dev = torch.device('cuda:0')
    work = bench.CONFIGS['cfg3'](dev, 0, graph=False, bf16=args.dtype == 'bf16')
    for _ in range(3):
        work.eager_step()
    torch.cuda.synchronize()
    p = work.plan
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


if __name__ == '__main__':
    main()
