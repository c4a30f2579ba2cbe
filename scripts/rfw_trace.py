"""Per-workgroup phase timeline of mep_rfw_epi_fwd (development build -DMEP_RFW_TRACE, via MEP_LIB)
on the cfg2 realformer plan: median shader-clock cycles per phase."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()


def main():
    import bench
    from mep_amd import _lib
    from mep_amd._lib import launch
    dev = torch.device('cuda:0')
    work = bench.Cfg2(dev, 0, graph=False)
    for _ in range(3):
        work.eager_step()
    p = work.plan
    L = _lib.lib()
    n = p.t_epif[0]
    tr = torch.zeros(16 * n, dtype=torch.int64, device=dev)
    L.mep_rfw_set_trace(ctypes.c_void_p(tr.data_ptr()))
    names = ['params', 'xp', 'xchg1', 'LN1', 'f1', 'xchg2', 'f', 'xchg3', 'LN2+st', 'drain']
    for rep in range(3):
        launch('mep_wsplit', p.d_wsplit, p.t_wsplit)
        launch('mep_rfw_epi_fwd', p.d_epi[0], n, extra=(p.spec.D, p.spec.FD))
        torch.cuda.synchronize()
        t = tr.view(n, 16).cpu().double()
        ph = [(t[:, k + 1] - t[:, k]) for k in range(10)]
        print('rep %d phases (median cycles): ' % rep + '  '.join('%s %.0f' % (nm, float(x.median())) for nm, x in zip(names, ph)))
        tot = t[:, 10] - t[:, 0]
        rt = t[:, 13]
        print('   total median %.0f cyc, max %.0f; start spread (realtime 100MHz) %.2f us; end spread %.2f us'
              % (float(tot.median()), float(tot.max()), float((rt - rt.min()).max()) / 100 - float(tot.max()) / 2.4e3, 0.0))
    L.mep_rfw_set_trace(ctypes.c_void_p(0))


if __name__ == '__main__':
    main()
