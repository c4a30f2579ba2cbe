"""Oracle for the Ren-MME ``Base_model`` family (TEST INFRASTRUCTURE ONLY).

Restates Ren-MME/run.py:157-340.  Same tri-modal structure as cmu-mosei with: one LayerNorm
shared by the three unify projections (run.py:164-166), the block LayerNorm named ``norm2``
(run.py:176,213), dropout(DROP) at ``proj`` and after the LayerNorm (run.py:209,213), 9 classes,
``norm3`` + ``out`` 18->9 in the head (run.py:279-292), and the R-Drop loss (run.py:331-334).
Dropout is an explicit callable so parity runs can pass identity (eval / p = 0).
"""
import torch

from . import common
from .cmu_mosei import multi_attn


def base_model(P, inputs, n_heads=8, n_layers=1, dropout=None):
    """Base_model.forward (Ren-MME/run.py:281-292).  ``inputs`` is the reference's 12-tuple
    (pre_text_feat, pre_text_mask, pro_text_feat, pro_text_mask, pre_video_feat, pre_video_mask,
    pro_video_feat, pro_video_mask, pre_audio_feat, pre_audio_mask, pro_audio_feat,
    pro_audio_mask)."""
    (ptf, ptm, qtf, qtm, pvf, pvm, qvf, qvm, paf, pam, qaf, qam) = inputs
    kw = dict(n_heads=n_heads, n_layers=n_layers, norm='norm2', unify_norm='norm1', dropout=dropout)
    last = multi_attn(P, 'intensity.', ptf, pvf, paf, ptm, pvm, pam, **kw)
    this = multi_attn(P, 'stimulation.', qtf, qvf, qaf, qtm, qvm, qam, **kw)
    y = common.bilinear_transfer(this, last, P['trans'])
    y = torch.cat([this, common.layer_norm(y, P['norm3.weight'], P['norm3.bias'])], dim=1)
    return common.linear(y, P['out.weight'], P['out.bias'])


def loss_fn(logits, labels, rdrop=True):
    """multi_loss (Ren-MME/run.py:295-304) + R-Drop KL (run.py:332-334)."""
    loss = common.circle_loss(logits, labels).mean()
    if rdrop:
        loss = loss + common.rdrop_kl(logits)
    return loss


def train_step(P, opt, inputs, labels, n_heads=8, n_layers=1, clip=1.0, dropout=None):
    """One Ren-MME ``train`` iteration (run.py:313-337)."""
    for p in P.values():
        p.grad = None
    logits = base_model(P, inputs, n_heads, n_layers, dropout)
    loss = loss_fn(logits, labels)
    loss.backward()
    total = common.clip_grad_norm([p.grad for p in P.values()], clip)
    opt.step()
    return loss.detach(), logits.detach(), total
