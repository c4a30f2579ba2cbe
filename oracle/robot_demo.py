"""Oracle for robot_demo.py inference (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates robot_demo.py:293-441 and 594-622: the 5-input biased k=1 Conv1d unify (text 768 -> D,
three visual streams 256 / 512 / 1024 -> D/3 each, concatenated in that order, audio 40 -> D),
learned position embeddings, the realformer-style residual block (identical arithmetic to
others/realformer.py's, oracle/realformer.block; with D = 192 and 6 heads the head dim is 32),
every layer's output of the nine chains concatenated per modality, mean + max pool over time,
the classifier on the pooled vector, the 4-model ensemble mean and demo_output's sigmoids.
"""
import math

import torch

from . import common
from .cmu_mosei import CHAINS, TIME_ORDER
from .realformer import block

EMOTIONS = ('happy', 'sad', 'angry', 'disgust', 'surprise', 'fear')
THRESHOLDS = (0.1, 0.1, -0.1, 0.0, 0.1, 0.0)   # robot_demo.py:609


def conv1(x, P, name):
    """nn.Conv1d(kernel_size=1) over the feature axis (robot_demo.py:296-308)."""
    return common.linear(x, P[name + '.weight'][:, :, 0], P[name + '.bias'])


def unify_pos(P, l, v256, v512, v1024, a):
    """Unify_Dimension_Conv1d (dropout inactive in eval) + Position_Embedding (robot_demo.py:302-321,
    391-394)."""
    u = 'unify_dimension.'
    v = torch.cat([conv1(v256, P, u + 'visual_256'), conv1(v512, P, u + 'visual_512'),
                   conv1(v1024, P, u + 'visual_1024')], dim=2)
    out = {}
    for m, x, name in (('l', conv1(l, P, u + 'linguistic'), 'linguistic'), ('v', v, 'visual'),
                       ('a', conv1(a, P, u + 'acoustic'), 'acoustic')):
        pos = P['%s_position.position_embeddings.weight' % name]
        out[m] = x + pos[: x.shape[1]].unsqueeze(0)
    return out


def multi_class(P, l, v256, v512, v1024, a, lm, vm, am, n_heads=6, n_layers=2):
    """Multi_class.forward (robot_demo.py:390-441) -> logits [B, 7]."""
    feats = unify_pos(P, l, v256, v512, v1024, a)
    masks = {'l': lm, 'v': vm, 'a': am}
    outs = {m: [] for m in 'lva'}
    for j, (qm, km) in enumerate(CHAINS):
        x, s = feats[qm], None
        for i in range(n_layers):
            x, s = block(P, 'multimodal_blocks.%d.' % (n_layers * j + i), x, feats[km], masks[km], n_heads, s)
            outs[qm].append(x)
    x = torch.cat([torch.cat(outs[m], dim=2) for m in TIME_ORDER], dim=1)
    return common.linear(common.mean_max_pool(x), P['classifier.weight'], P['classifier.bias'])


def ensemble(preds):
    """(pred_1 + pred_2 + pred_3 + pred_4) / 4 (robot_demo.py:550, 615)."""
    total = preds[0]
    for p in preds[1:]:
        total = total + p
    return total / len(preds)


def probabilities(pred_row):
    """demo_output's sigmoids(pred[0][c], t_c) = 1 / (1 + exp(-x + t)) (robot_demo.py:594-595, 617-622)."""
    return [1.0 / (1.0 + math.exp(-float(pred_row[c]) + THRESHOLDS[c])) for c in range(6)]
