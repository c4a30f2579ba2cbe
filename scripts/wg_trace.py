"""Phase trace of the weight-gradient launch (development builds with -DMEP_WG_TRACE, csrc/gemm.hip):
    MEP_LIB=variants/trace/lib.so python scripts/wg_trace.py [--dtype bf16] [--fold 0]
Runs the cfg3 bench plan's step eagerly, then the weight-gradient launch alone (fused, or the
two-launch form with --fold 0) and prints, over the workgroups, the spread of each phase's start
(0 start, 1 main loop, 2 main loop end, 3 slot written, 4 ticket drawn, 5 reducer end, 7 job workgroup done) relative to the
earliest workgroup start, in microseconds (100 MHz real-time counter)."""
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
    ap.add_argument('--fold', type=int, default=1)
    args = ap.parse_args()
    import bench
    from mep_amd import _lib, trimodal
    from mep_amd._lib import launch
    trimodal.WGRAD_FOLD = bool(args.fold)
    dev = torch.device('cuda:0')
    work = bench.CONFIGS['cfg3'](dev, 0, graph=False, bf16=args.dtype == 'bf16')
    for _ in range(3):
        work.eager_step()
    torch.cuda.synchronize()
    p = work.plan
    L = _lib.lib()
    fn = L.mep_wg_trace_read
    fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
    buf = np.zeros((8192, 8), dtype=np.uint64)
    for rep in range(3):
        fn(buf.ctypes.data)
        buf[:] = 0
        # clear the device copy: write zeros by a fresh read after a launch that stamps everything
        if args.fold:
            trimodal.wgrad_fused(p.d_wgrad, p.t_wgrad, p.d_colsum, p.t_colsum, p.head, p.head_grads,
                                 (None, None, None), None)
        else:
            launch('mep_wgrad', p.d_wgrad, p.t_wgrad)
        torch.cuda.synchronize()
        fn(buf.ctypes.data)
    nwg = p.t_wgrad
    jobs = trimodal.fold_job_wg(trimodal.fold_jobs(p.d_colsum.n, p.t_colsum, p.head), nwg, args.dtype == 'bf16') if args.fold else 0
    t = buf[:nwg + jobs].astype(np.float64)
    t0 = t[:, 0][t[:, 0] > 0].min()
    us = np.where(t > 0, (t - t0) / 100.0, np.nan)
    print('workgroups %d (+%d job workgroups), span %.2f us' % (nwg, jobs, np.nanmax(us[:, 5] if args.fold else us[:nwg, 3])))
    names = ['start', 'loop', 'loop end', 'slot written', 'ticket', 'end']
    for k, nm in enumerate(names):
        col = us[:nwg, k]
        if np.all(np.isnan(col)):
            continue
        q = np.nanpercentile(col, [0, 10, 50, 90, 100])
        print('  %-13s ' % nm + ' '.join('%7.2f' % v for v in q))
    if args.fold:
        red = ~np.isnan(us[:nwg, 5]) & (us[:nwg, 5] - us[:nwg, 4] > 0.3)
        d = us[:nwg, 5] - us[:nwg, 4]
        print('  reducer time (ticket -> end), %d reducers: ' % int(red.sum()) +
              ' '.join('%6.2f' % v for v in np.nanpercentile(d[red], [0, 50, 90, 100])))
        for k, nm in ((6, 'ticket -> first loads'),):
            d = us[:nwg, k] - us[:nwg, 4]
            print('  %s: ' % nm + ' '.join('%6.2f' % v for v in np.nanpercentile(d[red], [0, 50, 90, 100])))
        w = us[:nwg, 4] - us[:nwg, 3]
        print('  drain + ticket: ' + ' '.join('%6.2f' % v for v in np.nanpercentile(w, [0, 50, 90, 100])))
        if jobs:
            j = us[nwg:nwg + jobs]
            print('  job workgroups start %s done %s' % (
                ' '.join('%6.2f' % v for v in np.nanpercentile(j[:, 0], [0, 50, 100])),
                ' '.join('%6.2f' % v for v in np.nanpercentile(j[:, 7], [0, 50, 100]))))


if __name__ == '__main__':
    main()
