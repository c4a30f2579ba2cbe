import sys, torch
sys.path.insert(0, '/root/repo')
import mep_import; mep_import.load()
from tests.golden import fixtures
from tests.test_gpu_realformer import _state, _batch
meta, gold = fixtures.load('rf_state_small')
dev = torch.device('cuda:0')
m = _state(meta, dev)
l, v, a, labels, lm, vm, am, um = _batch(meta, dev)
out = m(l, v, a, lm, vm, am).detach().cpu()
want = torch.as_tensor(gold['logits'])
pad = ~um.bool().cpu()
print('padded slots', int(pad.sum()), 'max diff', float((out[pad] - want[pad]).abs().max()), 'max |want|', float(want.abs().max()))
print('real max diff', float((out[~pad] - want[~pad]).abs().max()))
