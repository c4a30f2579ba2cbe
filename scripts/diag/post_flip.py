"""Diagnose a post-step parameter mismatch of test_base_model_engine_step: the worst elements,
their reference gradients and the tensor's gradient scale."""
import sys
import torch
sys.path.insert(0, ".")
import mep_import  # noqa: E402
mep_import.load()
from tests.golden import fixtures
from tests.gpu_util import ren_model
from tests.test_gpu_ren import _batch
from mep_amd import ren_mme
from mep_amd.engine import TrainEngine
from mep_amd.optim import FusedAdamW

name = sys.argv[1] if len(sys.argv) > 1 else 'ren_small'
cuda = torch.device('cuda:0')
meta, gold = fixtures.load(name)
print('steps', meta['steps'])
model = ren_model(meta, cuda)
model.train()
opt = FusedAdamW(model, lr=1e-3)
eng = TrainEngine(model, opt, clip=1.0, rdrop=True, graph=False)
args, labels = _batch(meta, cuda)
packed = ren_mme._pack(args)
eng.step(*packed, labels)
torch.cuda.synchronize()
fl = model.mep_runner(cuda).flat
print([k for k in gold.keys()][:6])
for k, p in model.named_parameters():
    if 'grad/' + k not in gold:
        continue
    g = fl.view(fl.grad, k).detach().double().cpu().reshape(-1)
    w = torch.as_tensor(gold['grad/' + k]).double().reshape(-1)
    post = (p.detach().double().cpu().reshape(-1) - torch.as_tensor(gold['post/' + k]).double().reshape(-1)).abs()
    if float(post.max()) > 2e-5:
        ip = int(torch.argmax(post))
        print('POST', k, 'elem', ip, 'post err %.3e grad got %.6e want %.6e' % (float(post[ip]), float(g[ip]), float(w[ip])))
    e = (g - w).abs()
    i = int(torch.argmax(e / (w.abs() + 1e-12 * w.abs().max())))
    if k.endswith('unify_dimension.visual.weight') or float((e / (w.abs().max())).max()) > 1e-5:
        small = (w.abs() < 1e-4 * w.abs().max())
        print(k, 'max|g| %.3e  worst rel elem %d got %.6e want %.6e  max err/max %.2e  n(|g|<1e-4 max)=%d'
              % (float(w.abs().max()), i, float(g[i]), float(w[i]), float(e.max() / w.abs().max()), int(small.sum())))
        j = torch.argsort(w.abs())[:5]
        for jj in j.tolist():
            print('   small elem', jj, 'got %.4e want %.4e' % (float(g[jj]), float(w[jj])))
