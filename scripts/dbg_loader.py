import sys, numpy as np, torch, random
sys.path.insert(0, '/root/repo')
import mep_import; mep_import.load()
from tests.test_batching import _train_data
from tests.golden import fixtures
from mep_amd import batching, cmu_mosei
from mep_amd.optim import FusedAdamW
from tests.gpu_util import cmu_model
from oracle import batching as ob
cuda = torch.device('cuda')
meta, _ = fixtures.load('cmu_cfg1')
data, labels, pairs = _train_data(np.random.default_rng(4))
lens = (50, 50, 50)
store = batching.FeatureStore(data, cuda)
random.seed(3)
order = list(pairs); random.shuffle(order)
host = [list(zip(*ob.cmu_batch(data, labels, order[i:i + 16], lens))) for i in range(0, len(order), 16)]
random.seed(3)
dev = list(batching.cmu_data_loader(store, lens)(list(pairs), labels, 16))
print(len(host), len(dev), type(dev[0]))
# compare assembled tensors
for bi, (h, d) in enumerate(zip(host, dev)):
    ht = [torch.tensor(np.array(x)) for x in h]
    dt = d.tensors() if hasattr(d, 'tensors') else None
    print(bi, [tuple(t.shape) for t in ht][:3], type(d))
    break
m1 = cmu_model(meta, cuda); m1.train()
m2 = cmu_model(meta, cuda); m2.train()
for name, m in (('host', m2),):
    pass
# same batch twice through a fresh model: determinism
for trial in range(2):
    m = cmu_model(meta, cuda); o = FusedAdamW(m, lr=1e-3)
    l = cmu_mosei.train(m, host[:1], o)
    print('host batch0 loss', trial, repr(l))
for trial in range(2):
    m = cmu_model(meta, cuda); o = FusedAdamW(m, lr=1e-3)
    random.seed(3)
    l = cmu_mosei.train(m, list(batching.cmu_data_loader(store, lens)(list(pairs), labels, 16))[:1], o)
    print('dev batch0 loss', trial, repr(l))
