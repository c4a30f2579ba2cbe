"""Time mep_wgrad of the cfg3 plan under different segmentations (development aid)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()


def main():
    import bench
    from mep_amd import trimodal
    from mep_amd._lib import launch
    dev = torch.device('cuda:0')
    work = bench.Cfg3(dev, 0, graph=False)
    work.eager_step()
    p = work.plan
    from mep_amd import trimodal as tm
    cases = [('bal%d' % n, dict(n_wg=n)) for n in (128, 160, 192, 200, 208, 224, 240, 256)]
    cases += [('tps%d' % t, dict(tok_per_split=t)) for t in (1072, 1000, 900)]
    for name, kw in cases:
        if 'n_wg' in kw:
            tm.WG_TARGET_OVERRIDE = kw.pop('n_wg')
        ws, arr, n_wg, rmax = trimodal.make_wgrad(p._wgrad_items, dev, **kw)
        for _ in range(3):
            launch('mep_wgrad', arr, n_wg)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            launch('mep_wgrad', arr, n_wg)
        b.record()
        torch.cuda.synchronize()
        print('%-10s wgs %4d  %.2f us' % (name, n_wg, a.elapsed_time(b) * 1e3 / 50), flush=True)


if __name__ == '__main__':
    main()
