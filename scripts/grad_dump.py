"""Development aid: one State_Transfer plan forward + backward (fixed seed) -> logits and the flat
gradient saved to argv[1]; run under two MEP_LIB builds and compare (--cmp a b: bitwise)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(path):
    import mep_import
    mep_import.load()
    from mep_amd import realformer as rf
    from mep_amd import rf_plan
    cuda = torch.device('cuda:0')
    B, P, T = 13, 5, 50
    torch.manual_seed(7)
    st = rf.State_Transfer(300, 35, 74, 96, T, T, T, 6, 2, 2).to(cuda)
    runner = st.mep_runner(cuda)
    feats = tuple(torch.randn(B, P, T, d, device=cuda) for d in (300, 35, 74))
    masks = tuple((torch.rand(B, P, T, device=cuda) > 0.2).float() for _ in range(3))
    dout = torch.randn(B, P, 6, device=cuda)
    plan = rf_plan.RealformerPlan(runner.spec, runner.flat, B, P, cuda)
    plan.set_inputs(*feats, *masks)
    plan.forward(grad=True)
    runner.flat.grad.zero_()
    plan.backward(ext_dout=dout)
    torch.cuda.synchronize()
    torch.save({'out': plan.out.cpu(), 'grad': runner.flat.grad.cpu()}, path)


def cmp(a, b):
    x, y = torch.load(a), torch.load(b)
    for k in x:
        d = (x[k] - y[k]).abs()
        print(k, 'equal' if torch.equal(x[k], y[k]) else 'DIFF max %.3g n %d' % (d.max().item(), int((d > 0).sum())),
              'finite' if torch.isfinite(x[k]).all() else 'NONFINITE')


if __name__ == '__main__':
    if sys.argv[1] == '--cmp':
        cmp(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
