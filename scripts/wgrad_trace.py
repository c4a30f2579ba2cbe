"""Per-workgroup timeline of mep_wgrad (development build with -DMEP_WG_TRACE, via MEP_LIB)."""
import collections
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
    from mep_amd import _lib, trimodal
    from mep_amd._lib import launch
    dev = torch.device('cuda:0')
    work = bench.Cfg3(dev, 0, graph=False)
    work.eager_step()
    p = work.plan
    L = _lib.lib()
    for name, kw in (('balanced', {}), ('tps1072', dict(tok_per_split=1072))):
        ws, arr, n_wg, rmax = trimodal.make_wgrad(p._wgrad_items, dev, **kw)
        tr = torch.zeros(8 * n_wg, dtype=torch.int64, device=dev)
        L.mep_wgrad_set_trace(ctypes.c_void_p(tr.data_ptr()))
        for _ in range(3):
            launch('mep_wgrad', arr, n_wg)
        torch.cuda.synchronize()
        t = tr.view(n_wg, 8).cpu()
        t0 = int(t[:, 0].min())
        dur = (t[:, 4] - t[:, 0]).double() / 100.0     # s_memrealtime: 100 MHz -> us
        start = (t[:, 0] - t0).double() / 100.0
        end = (t[:, 4] - t0).double() / 100.0
        ph = [(t[:, k + 1] - t[:, k]).double() / 100.0 for k in range(4)]
        print('%s phases (median us): setup %.2f  main loop %.2f  reduce+write %.2f  tail %.2f; k blocks (wave 0) median %d'
              % (name, *[float(x.median()) for x in ph], int(t[:, 7].median())), flush=True)
        cu = [(int(x) >> 8) & 15 | ((int(x) >> 12) & 1) << 4 | ((int(x) >> 13) & 7) << 5 for x in t[:, 5]]
        key = [(int(t[i, 6]) & 15, cu[i]) for i in range(n_wg)]
        per = collections.Counter(key)
        print('%s: wgs %d  span %.1f us  dur min %.1f med %.1f max %.1f  start max %.1f  distinct CUs %d  max WGs/CU %d'
              % (name, n_wg, float(end.max()), float(dur.min()), float(dur.median()), float(dur.max()),
                 float(start.max()), len(per), max(per.values())), flush=True)
        late = sorted(range(n_wg), key=lambda i: -float(end[i]))[:6]
        print('   latest:', [(i, round(float(start[i]), 1), round(float(dur[i]), 1)) for i in late])
        # per-workgroup record for cost fitting: duration and (MT, KT of the column group, tokens) per segment
        items = [tuple(it) + (0,) * (5 - len(it)) for it in p._wgrad_items]
        segs, _ = trimodal.wgrad_segments(items, tok_per_split=kw.get('tok_per_split'))
        with open(os.path.join(ROOT, 'gpurun_out', 'wgrad_trace_%s.txt' % name), 'w') as f:
            for i, b in enumerate(segs):
                parts = []
                for (it, cg, t0, t1, sl) in b:
                    N = items[it][1]
                    ktot = sum(x[1] for x in items[it][3])
                    mt, kt, ncg = trimodal.wgrad_geometry(N, ktot)
                    parts.append('%d,%d,%d' % (mt, min(kt, -(-ktot // 32) - cg * kt), t1 - t0))
                f.write('%.2f %s\n' % (float(dur[i]), ' '.join(parts)))
        L.mep_wgrad_set_trace(ctypes.c_void_p(0))


if __name__ == '__main__':
    main()
