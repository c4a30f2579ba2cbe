"""Development aid: which State_Transfer plan buffers differ between the weight-stationary
epilogues (MEP_RFS=1) and the per-tile kernels (MEP_RFS=0) after one forward + backward."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mep_import  # noqa: E402

mep_import.load()


def main():
    from mep_amd import realformer as rf
    from mep_amd import rf_plan
    cuda = torch.device('cuda:0')
    B, P, T = 16, 6, 50
    torch.manual_seed(B * P)
    st = rf.State_Transfer(300, 35, 74, 96, T, T, T, 6, 2, 2).to(cuda)
    runner = st.mep_runner(cuda)
    feats = tuple(torch.randn(B, P, T, d, device=cuda) for d in (300, 35, 74))
    masks = tuple((torch.rand(B, P, T, device=cuda) > 0.2).float() for _ in range(3))
    dout = torch.randn(B, P, 6, device=cuda)
    snaps = []
    for on in ('1', '0'):
        os.environ['MEP_RFS'] = on
        plan = rf_plan.RealformerPlan(runner.spec, runner.flat, B, P, cuda)
        plan.set_inputs(*feats, *masks)
        plan.forward(grad=True)
        torch.cuda.synchronize()
        fwd = {('fwd', j, k): v.clone() for j, b in enumerate(plan.blocks) for k, v in b.items() if torch.is_tensor(v)}
        runner.flat.grad.zero_()
        plan.backward(ext_dout=dout)
        torch.cuda.synchronize()
        snap = {('bwd', j, k): v.clone() for j, b in enumerate(plan.blocks) for k, v in b.items() if torch.is_tensor(v)}
        snap.update(fwd)
        snap[('grad',)] = runner.flat.grad.clone()
        snaps.append(snap)
    for k in sorted(snaps[0], key=str):
        a, b = snaps[0][k], snaps[1][k]
        if a.shape != b.shape or not torch.equal(a, b):
            d = (a.float() - b.float()).abs()
            idx = int(d.reshape(-1).argmax())
            print('DIFF', k, tuple(a.shape), 'max %.3g at flat %d (of %d), n_diff %d' % (d.max().item(), idx, d.numel(), int((d > 0).sum())))
    print('compared', len(snaps[0]))


if __name__ == '__main__':
    main()
