"""Oracle for the others/realformer.py ``State_Transfer`` family (TEST INFRASTRUCTURE ONLY).

Restates others/realformer.py:133-318: k=1 Conv1d unify (== bias-free Linear on the feature
axis), learned position embeddings, the RealFormer block with Q/K/V projections, ReZero-style
scalars ``a``/``b``, FFN and two post-LayerNorms, the ``Multi_class`` pooled encoder and the
sigmoid-gated ``State_Transfer`` recurrence over the P utterances.
"""
import torch

from . import common
from .cmu_mosei import CHAINS, TIME_ORDER


def block(P, pre, q, kv, mask, n_heads, s_prev=None):
    """Attention_Block.forward (realformer.py:182-209)."""
    qp = common.linear(q, P[pre + 'w_qkv.0.weight'])
    kp = common.linear(kv, P[pre + 'w_qkv.1.weight'])
    vp = common.linear(kv, P[pre + 'w_qkv.2.weight'])
    x, s = common.residual_attention(qp, kp, vp, mask, n_heads, c=P[pre + 'c'], s_prev=s_prev)
    x = common.linear(x, P[pre + 'proj.weight'])
    h = common.layer_norm(q + P[pre + 'a'] * x, P[pre + 'norm1.weight'], P[pre + 'norm1.bias'])
    f = common.linear(torch.relu(common.linear(h, P[pre + 'ffn.0.weight'], P[pre + 'ffn.0.bias'])),
                      P[pre + 'ffn.2.weight'], P[pre + 'ffn.2.bias'])
    return common.layer_norm(h + P[pre + 'b'] * f, P[pre + 'norm2.weight'], P[pre + 'norm2.bias']), s


def encode_chain(P, pre, x, n_layers, n_heads, mask, first_block=0, kv=None):
    """Run ``n_layers`` consecutive blocks of one chain starting at block ``first_block`` (the
    cfg2 "text chain": multimodal_blocks[0..1] over l, realformer.py:232-233)."""
    kv = x if kv is None else kv
    s = None
    for i in range(n_layers):
        x, s = block(P, pre + 'multimodal_blocks.%d.' % (first_block + i), x, kv, mask, n_heads, s)
    return x, s


def unify_pos(P, pre, l, v, a):
    """Unify_Dimension_Conv1d + Position_Embedding add (realformer.py:133-152,224-227)."""
    out = {}
    for m, x, name in (('l', l, 'linguistic'), ('v', v, 'visual'), ('a', a, 'acoustic')):
        w = P[pre + 'unify_dimension.%s.weight' % name][:, :, 0]
        pos = P[pre + '%s_position.position_embeddings.weight' % name]
        out[m] = common.linear(x, w) + pos[: x.shape[1]].unsqueeze(0)
    return out


def multi_class(P, pre, l, v, a, lm, vm, am, n_heads=6, n_layers=2):
    """Multi_class.forward (realformer.py:223-264) -> [B, D]."""
    feats = unify_pos(P, pre, l, v, a)
    masks = {'l': lm, 'v': vm, 'a': am}
    last = {}
    for j, (qm, km) in enumerate(CHAINS):
        x, _ = encode_chain(P, pre, feats[qm], n_layers, n_heads, masks[km], n_layers * j, feats[km])
        last[(qm, km)] = x
    grouped = {qm: torch.cat([last[(qm, km)] for (q2, km) in CHAINS if q2 == qm], dim=2) for qm in 'lva'}
    x = torch.cat([grouped[m] for m in TIME_ORDER], dim=1)
    x = common.linear(common.mean_max_pool(x), P[pre + 'fully_connected.weight'], P[pre + 'fully_connected.bias'])
    return torch.relu(common.layer_norm(x, P[pre + 'normalization.weight'], P[pre + 'normalization.bias']))


def state_transfer(P, l, v, a, lm, vm, am, n_heads=6, n_layers=2):
    """State_Transfer.forward (realformer.py:272-286): shared encoder per utterance, then the
    sigmoid/tanh gate.  Inputs [B, P, T, d]; returns [B, P, 6]."""
    outs, gates = [], []
    for i in range(l.shape[1]):
        f = multi_class(P, 'feature.', l[:, i], v[:, i], a[:, i], lm[:, i], vm[:, i], am[:, i], n_heads, n_layers)
        o, g = common.linear(f, P['classifier.weight'], P['classifier.bias']).chunk(2, 1)
        if i:
            alpha = torch.sigmoid(g + gates[-1])
            o = (1 - alpha) * o + alpha * torch.tanh(torch.matmul(outs[-1], P['trans']))
        outs.append(o)
        gates.append(g)
    return torch.stack(outs, dim=1)


def loss_fn(out, labels, utt_mask):
    """(circle_loss * mask).mean() over B*P (realformer.py:311-312)."""
    return (common.circle_loss(out, labels) * utt_mask).mean()


def train_step(P, opt, batch, n_heads=6, n_layers=2, clip=1.0):
    """One realformer ``train`` iteration (realformer.py:306-315), Adam without weight decay."""
    for p in P.values():
        p.grad = None
    l, v, a, labels, lm, vm, am, um = batch
    out = state_transfer(P, l, v, a, lm, vm, am, n_heads, n_layers)
    loss = loss_fn(out, labels, um)
    loss.backward()
    total = common.clip_grad_norm([p.grad for p in P.values()], clip)
    opt.step()
    return loss.detach(), out.detach(), total
