"""Oracle for the cmu-mosei ``Concat_Trans`` family (TEST INFRASTRUCTURE ONLY).

Restates cmu-mosei/run.py:206-390 as functions over a state_dict-keyed parameter dict.
The Ren-MME ``Base_model`` shares this structure; its differences (shared unify LayerNorm,
``norm2``/``norm3`` names, dropout, 9 classes) are handled by the ``variant`` argument and
live in oracle/ren_mme.py.
"""
import torch

from . import common

# The nine cross-modal chains in block order (cmu-mosei/run.py:279-313):
# (query modality, key/value modality); chains 0-2 feed the l rows, 3-5 the v rows, 6-8 the a rows.
CHAINS = (('l', 'l'), ('l', 'v'), ('l', 'a'),
          ('v', 'v'), ('v', 'l'), ('v', 'a'),
          ('a', 'a'), ('a', 'l'), ('a', 'v'))
# time-axis concatenation order of the pooled tensor: [l rows, a rows, v rows]  (run.py:317)
TIME_ORDER = ('l', 'a', 'v')


def unify(P, pre, l, v, a, shared_norm=None):
    """Unify_Dimension (cmu-mosei/run.py:207-214); Ren-MME adds one shared LayerNorm
    (Ren-MME/run.py:158-166)."""
    out = {'l': common.linear(l, P[pre + 'unify_dimension.linguistic.weight']),
           'v': common.linear(v, P[pre + 'unify_dimension.visual.weight']),
           'a': common.linear(a, P[pre + 'unify_dimension.acoustic.weight'])}
    if shared_norm is not None:
        w, b = P[pre + 'unify_dimension.' + shared_norm + '.weight'], P[pre + 'unify_dimension.' + shared_norm + '.bias']
        out = {k: common.layer_norm(x, w, b) for k, x in out.items()}
    return out


def block(P, pre, q, kv, mask, n_heads, s_prev=None, norm='norm1', dropout=None):
    """Attention_Block.forward (cmu-mosei/run.py:236-262): attention without a QKV projection,
    ``proj``, ``cat([q, x])``, ``minus`` (2D->D), LayerNorm.  ``dropout`` is a callable applied
    where the reference applies ``self.drop`` (identity for cmu-mosei, DROP = 0)."""
    drop = dropout or (lambda t: t)
    x, s = common.residual_attention(q, kv, kv, mask, n_heads, c=P[pre + 'c'], s_prev=s_prev)
    x = drop(common.linear(x, P[pre + 'proj.weight']))
    y = common.linear(torch.cat([q, x], dim=-1), P[pre + 'minus.weight'])
    y = drop(common.layer_norm(y, P[pre + norm + '.weight'], P[pre + norm + '.bias']))
    return y, s


def multi_attn(P, pre, l, v, a, lm, vm, am, n_heads, n_layers, norm='norm1', unify_norm=None,
               dropout=None):
    """Multi_ATTN.forward (cmu-mosei/run.py:272-319).  Returns classifier logits."""
    feats = unify(P, pre, l, v, a, unify_norm)
    masks = {'l': lm, 'v': vm, 'a': am}
    rows = {'l': [], 'v': [], 'a': []}
    for j, (qm, km) in enumerate(CHAINS):
        x, s = feats[qm], None
        for i in range(n_layers):
            x, s = block(P, pre + 'multimodal_blocks.%d.' % (n_layers * j + i), x, feats[km],
                         masks[km], n_heads, s_prev=s, norm=norm, dropout=dropout)
            rows[qm].append(x)
    x = torch.cat([torch.cat(rows[m], dim=2) for m in TIME_ORDER], dim=1)
    return common.linear(common.mean_max_pool(x), P[pre + 'classifier.weight'])


def concat_trans(P, l, v, a, lm, vm, am, n_heads=6, n_layers=1):
    """Concat_Trans.forward (cmu-mosei/run.py:329-339).  Inputs carry the (prev, cur) utterance
    pair on axis 1: l [B,2,T,300] etc.; masks [B,2,T]."""
    last = multi_attn(P, 'intensity.', l[:, 0], v[:, 0], a[:, 0], lm[:, 0], vm[:, 0], am[:, 0],
                      n_heads, n_layers)
    this = multi_attn(P, 'stimulation.', l[:, 1], v[:, 1], a[:, 1], lm[:, 1], vm[:, 1], am[:, 1],
                      n_heads, n_layers)
    y = common.bilinear_transfer(this, last, P['trans'])
    y = torch.cat([this, common.layer_norm(y, P['norm1.weight'], P['norm1.bias'])], dim=1)
    return common.linear(y, P['out.weight'], P['out.bias'])


def loss_fn(logits, labels):
    """``multi_circle_loss(...).mean()`` (cmu-mosei/run.py:365-366)."""
    return common.circle_loss(logits, labels).mean()


def train_step(P, opt, batch, n_heads=6, n_layers=1, clip=1.0):
    """One ``train`` iteration (cmu-mosei/run.py:360-369) on already-built tensors:
    zero_grad, forward, loss.mean, backward, clip_grad_norm_(clip), optimizer step.
    ``P`` maps names to leaf tensors with requires_grad; ``opt`` is a common.AdamState over
    them.  Returns (loss, logits, grad-norm-before-clip)."""
    for p in P.values():
        p.grad = None
    l, v, a, lm, vm, am, labels = batch
    logits = concat_trans(P, l, v, a, lm, vm, am, n_heads, n_layers)
    loss = loss_fn(logits, labels)
    loss.backward()
    names = list(P.keys())
    total = common.clip_grad_norm([P[k].grad for k in names], clip)
    opt.step()
    return loss.detach(), logits.detach(), total
