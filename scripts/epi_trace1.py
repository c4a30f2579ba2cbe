"""Per-workgroup timeline of the single-phase fp32 epilogue forward (epi_fwd_wp2r) at cfg3: kernel
start -> weights staged -> tiles done, from a development build with -DMEP_EPI_TRACE (MEP_LIB).
Prints the medians / maxima of both phases and the spread of the workgroups' start times."""
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
    n_wg = p.t_epi[0] * p.d_epi[0].n
    tr = torch.zeros(8 * n_wg, dtype=torch.int64, device=dev)
    L.mep_epi_set_trace(ctypes.c_void_p(tr.data_ptr()))
    for rep in range(4):
        tr.zero_()
        launch('mep_block_epi_fwd', p.d_epi[0], p.t_epi[0], threads=p.spec.D | p.prec)
        torch.cuda.synchronize()
        t = tr.view(n_wg, 8).cpu().double()
        t = t[t[:, 2] > 0]
        t0 = t[:, 0].min()
        st, stage, comp = (t[:, 0] - t0) / 100.0, (t[:, 1] - t[:, 0]) / 100.0, (t[:, 2] - t[:, 1]) / 100.0
        span = (t[:, 2].max() - t0).item() / 100.0
        q = lambda x: '%.2f / %.2f / %.2f' % (float(x.min()), float(x.median()), float(x.max()))  # noqa: E731
        print('rep %d: %d wgs, span %.1f us; start offset (min/med/max) %s; staging %s; tiles %s'
              % (rep, t.shape[0], span, q(st), q(stage), q(comp)))
        # wave 0's first tile: staged -> xp product done (3) -> z product done (4) -> LN + stores (5)
        ph = [(t[:, 3] - t[:, 1]) / 100.0, (t[:, 4] - t[:, 3]) / 100.0, (t[:, 5] - t[:, 4]) / 100.0]
        print('    wave 0 first tile: xp %s | z %s | LN + stores %s' % tuple(q(x) for x in ph))
        two = t[:, 7] > 0   # workgroups whose wave 0 ran a second tile
        if two.any():
            u = t[two]
            print('    wave 0 second tile (%d wgs): %s us; first tile of those: %s'
                  % (int(two.sum()), q((u[:, 7] - u[:, 6]) / 100.0), q((u[:, 5] - u[:, 1]) / 100.0)))
    L.mep_epi_set_trace(ctypes.c_void_p(0))


if __name__ == '__main__':
    main()
