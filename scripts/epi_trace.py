"""Per-workgroup phase timeline of mep_block_epi_fwd (development build with -DMEP_EPI_TRACE, via MEP_LIB)."""
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
    work = bench.Cfg3(dev, 0, graph=False)
    work.eager_step()
    p = work.plan
    L = _lib.lib()
    n_desc = p.d_epi[0].n
    n_wg = p.t_epi[0] * n_desc
    tr = torch.zeros(8 * n_wg, dtype=torch.int64, device=dev)
    L.mep_epi_set_trace(ctypes.c_void_p(tr.data_ptr()))
    for _ in range(3):
        launch('mep_block_epi_fwd', p.d_epi[0], p.t_epi[0], threads=p.spec.D | p.prec)
    torch.cuda.synchronize()
    t = tr.view(n_wg, 8).cpu()
    ok = t[:, 4] > 0
    t = t[ok]
    ph = [(t[:, k + 1] - t[:, k]).double() / 100.0 for k in range(4)]
    span = (t[:, 4].max() - t[:, 0].min()).item() / 100.0
    print('epi_fwd wgs %d  span %.1f us  phases (median / max us): stage Wp %.2f/%.2f  phase 1 %.2f/%.2f  '
          'stage Wm %.2f/%.2f  phase 2 %.2f/%.2f' % (int(ok.sum()), span, *[v for x in ph for v in (float(x.median()), float(x.max()))]))
    L.mep_epi_set_trace(ctypes.c_void_p(0))


if __name__ == '__main__':
    main()
