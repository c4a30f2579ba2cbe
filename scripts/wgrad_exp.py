"""Development timing of k_wgrad on subsets of the bench plan's weight-gradient items and with
different token splits.   python scripts/wgrad_exp.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()


def timeit(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    from bench import synth_batch
    from mep_amd import cmu_mosei, trimodal
    from mep_amd._lib import launch
    from mep_amd.engine import TrainEngine
    from mep_amd.optim import FusedAdamW
    dev = torch.device('cuda:0')
    model = cmu_mosei.Concat_Trans(dim=96, l_len=50, v_len=50, a_len=50, n_heads=6, n_layers=1, ffn=1).to(dev).train()
    eng = TrainEngine(model, FusedAdamW(model, lr=1e-3), graph=False)
    plan = model.mep_runner(dev).plan(64, (50, 50, 50))
    plan.set_inputs(*synth_batch(0, dev))
    eng.step_plan(plan)
    torch.cuda.synchronize()
    items = plan._wgrad_items
    subsets = {'all': items, 'blocks': items[:36], 'wp': items[0:36:2], 'wm': items[1:36:2], 'unify': items[36:],
               'unify_l': [items[36], items[39]], 'unify_va': [items[37], items[38], items[40], items[41]]}
    for n_wg in [int(x) for x in os.environ.get('NWG', '256,512,768,1024,1536').split(',')]:
        for name, its in subsets.items():
            tps = trimodal.wgrad_splits([tuple(i) + (0,) * (5 - len(i)) for i in its], n_wg)
            ws, arr, tmax, rmax = trimodal.make_wgrad(its, dev, tok_per_split=tps)
            t = timeit(lambda: launch('mep_wgrad', arr, tmax))
            tr = timeit(lambda: launch('mep_wgrad_reduce', arr, rmax))
            print('n_wg %5d %-9s wgs %4d  wgrad %8.2f us  reduce %7.2f us' % (n_wg, name, tmax, t, tr),
                  flush=True)

if __name__ == '__main__':
    main()
