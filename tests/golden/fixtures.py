"""Load golden fixtures and rebuild their inputs / parameters from the recorded seeds."""
import glob
import json
import os

import numpy as np
import torch

from . import specs

HERE = os.path.dirname(os.path.abspath(__file__))


def names(kind=None):
    out = []
    for p in sorted(glob.glob(os.path.join(HERE, '*.npz'))):
        n = os.path.basename(p)[:-4]
        with np.load(p) as z:
            if 'meta' not in z.files:      # data-only fixtures (batch_golden, eval_golden)
                continue
        if kind is None or load(n)[0]['kind'] == kind:
            out.append(n)
    return out


def load(name):
    z = np.load(os.path.join(HERE, name + '.npz'))
    meta = json.loads(str(z['meta']))
    return meta, {k: z[k] for k in z.files if k != 'meta'}


def params(meta, requires_grad=True, device='cpu'):
    vals = specs.param_values(meta['shapes'], meta['seed'], meta.get('overrides'))
    return {k: torch.tensor(v, device=device, requires_grad=requires_grad) for k, v in vals.items()}


def batch(meta):
    """Rebuild the recorded batch as CPU torch tensors in the reference's argument order."""
    fam, spec = meta['family'], meta['batch']
    if fam == 'cmu':
        return tuple(torch.from_numpy(x) for x in specs.cmu_batch(**spec))
    if fam == 'ren':
        inputs, labels = specs.ren_batch(**spec)
        return tuple(torch.from_numpy(x) for x in inputs), torch.from_numpy(labels)
    if fam == 'robot':
        return tuple(torch.from_numpy(x) for x in specs.robot_batch(**spec))
    return tuple(torch.from_numpy(x) for x in specs.realformer_batch(**spec))


def block_inputs(meta):
    D, H = meta['ctor']['dim'], meta['ctor']['n_heads']
    return specs.block_inputs(meta['seed'] + 1, meta['B'], meta['Tq'], meta['Tk'], D, H, meta['with_prev'],
                              meta.get('mask_kind', 'key'))


def chain_inputs(meta):
    rng = np.random.default_rng(meta['seed'] + 1)
    B, T = meta['B'], meta['T']
    lm = specs.masks_for(rng, (B,), T)
    x = specs.features(rng, (B, T, meta['consts']['L_DIM']), lm)
    G = rng.standard_normal((B, T, meta['ctor']['dim'])).astype(np.float32)
    return x, lm, G
