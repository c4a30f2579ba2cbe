"""GPU check of the pool-backward fold (MEP_POOL_FOLD): one eager Concat_Trans step with the fold
and without it on the same weights and batch; prints the largest difference of every block's
dZ / dX / dQ and of the flat gradient."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import mep_import  # noqa: E402

mep_import.load()
from mep_amd import cmu_mosei, trimodal  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(0)
B, T = 4, (6, 9, 11)
m = cmu_mosei.Concat_Trans(32, T[0], T[1], T[2], 2, int(sys.argv[1]) if len(sys.argv) > 1 else 1, 1).to(dev)
x = [torch.randn(B, 2, t, d, device=dev) for t, d in zip(T, (300, 35, 74))]
mk = [torch.ones(B, 2, t, device=dev) for t in T]
lab = (torch.rand(B, 7, device=dev) < 0.3).long()
res = {}
for fold in (False, True):
    trimodal.POOL_FOLD = fold
    p = trimodal.TriModalPlan(m.mep_runner(dev).spec, m.mep_runner(dev).flat, B, T, dev)
    p.set_inputs(x[0], x[1], x[2], mk[0], mk[1], mk[2], lab)
    m.mep_runner(dev).flat.grad.zero_()
    p.forward(grad=True)
    p.backward()
    torch.cuda.synchronize()
    if not fold:   # the formula the fold forms, against mep_pool_bwd's dXcat
        for e in range(2):
            dp, am = p.dpooled[e].view(B, 2, p.C), p.argmax[e].long()
            want = (dp[:, 0] / p.Ttot)[:, None, :].expand(B, p.Ttot, p.C).clone()
            hit = am[:, None, :] == torch.arange(p.Ttot, device=dev)[None, :, None]
            want = torch.where(hit, want + dp[:, 1][:, None, :], want)
            print('formula vs dXcat', e, float((want - p.dXcat[e]).abs().max()), float(p.dXcat[e].abs().max()))
    # block 0's dZ from its upstream gradient (LayerNorm backward in torch)
    b0 = p.blocks[0]
    e0, D = b0['e'], 32
    up = res[False][3][e0] if fold else p.dXcat[e0]
    g = up[:, p.toff[b0['qm']]:p.toff[b0['qm']] + b0['Tq'], b0['col']:b0['col'] + D].reshape(-1, D)
    w = p.flat.view(p.flat.buf, b0['pre'] + p.spec.block_norm + '.weight')
    st = b0['estat']
    xh = (b0['Z'] - st[:, :1]) * st[:, 1:]
    gw = g * w
    dz = st[:, 1:] * (gw - gw.mean(1, keepdim=True) - xh * (gw * xh).mean(1, keepdim=True))
    if fold:
        print('per-row diff', [round(float(x), 5) for x in (dz - b0['dZ']).abs().max(1).values[:24]])
        print('per-col diff', [round(float(x), 5) for x in (dz - b0['dZ']).abs().max(0).values])
    print('fold', fold, 'block0 dZ vs torch LN backward', float((dz - b0['dZ']).abs().max()), float(dz.abs().max()))
    res[fold] = ([{k: b[k].clone() for k in ('dZ', 'dX', 'dQ', 'dXP')} for b in p.blocks],
                 m.mep_runner(dev).flat.grad.clone(), [d.clone() for d in p.dpooled],
                 [x.clone() for x in p.dXcat] if p.dXcat is not None else None)
a, b = res[False], res[True]
print('dpooled', max(float((u - v).abs().max()) for u, v in zip(a[2], b[2])))
for i, (u, v) in enumerate(zip(a[0], b[0])):
    print(i, {k: float((u[k] - v[k]).abs().max()) for k in u})
print('grad', float((a[1] - b[1]).abs().max()), float(a[1].abs().max()))
