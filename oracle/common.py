"""Shared oracle arithmetic (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Everything is fp32 CPU PyTorch, written as plain functions over a parameter dict keyed by the
reference's state_dict names.  Each function cites the reference lines whose arithmetic it
restates; the order of floating-point operations follows the reference where it matters
(the residual-score / mask sequence, F7 in SURVEY.md).
"""
import math

import torch

MASK_BIG = 1.0e8       # cmu-mosei/run.py:253, others/realformer.py:200, Ren-MME/run.py:205
CIRCLE_BIG = 1.0e12    # cmu-mosei/run.py:344-345


def heads(x, n_heads):
    """[B, T, D] -> [B, H, T, D/H]  (split_last + transpose, cmu-mosei/run.py:226-231,242)."""
    b, t, d = x.shape
    return x.reshape(b, t, n_heads, d // n_heads).transpose(1, 2)


def merge(x):
    """[B, H, T, hd] -> [B, T, H*hd]  (transpose + merge_last, cmu-mosei/run.py:232-235,255-256)."""
    b, h, t, hd = x.shape
    return x.transpose(1, 2).reshape(b, t, h * hd)


def residual_attention(q, k, v, mask, n_heads, c=None, s_prev=None):
    """Residual scaled-dot-product attention, cmu-mosei/run.py:236-256 (== realformer.py:189-203).

    q [B,Tq,D], k/v [B,Tk,D] already projected (or raw features for cmu/Ren-MME), mask [B,Tk]
    or [B,Tq,Tk] (1 = keep; the 3-D form is shared by the heads, run.py:250-252) or None.
    Returns (x [B,Tq,D] before ``proj``, post-mask scores [B,H,Tq,Tk]).
    Op order: (q.k^T)/sqrt(hd)  [+ c*S_prev]  then  -= 1e8*(1-mask)   (run.py:243-253).
    """
    qh, kh, vh = heads(q, n_heads), heads(k, n_heads), heads(v, n_heads)
    scale = float(math.sqrt(kh.shape[-1]))
    s = torch.matmul(qh, kh.transpose(-2, -1)) / scale
    if s_prev is not None:
        s = s + c * s_prev
    if mask is not None:
        m = mask[:, None, None, :] if mask.dim() == 2 else mask[:, None, :, :]
        s = s - MASK_BIG * (1.0 - m)
    p = torch.softmax(s, dim=-1)
    return merge(torch.matmul(p, vh)), s


def layer_norm(x, w, b, eps=1e-5):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)


def linear(x, w, b=None):
    y = torch.matmul(x, w.t())
    return y if b is None else y + b


# Max-pool routing hook (test infrastructure: tests/test_gpu_bf16.py, make_bf16_budget.py).  A bf16
# execution picks different max-pool argmaxes than the fp32 one wherever two time steps are within
# bf16 noise, and one such flip moves a block's whole gradient: the bf16 checks compare against
# the fp32 arithmetic on the SAME routing.  POOL_ROUTE: None, or a list of [B, C] time indices
# consumed one per pool call (in call order: intensity, then stimulation); the max half of the pool
# then gathers x at those steps (and its gradient goes to them).  POOL_SEEN collects the indices
# every call used (torch.max's first-index tie rule when not routed).
POOL_ROUTE = None
POOL_SEEN = []
# with POOL_ROUTE: the largest accepted shortfall of a replayed step below the true max of its
# column, relative to the column's max |x| over time (None: unchecked).  A routing taken from a
# bf16 execution may pick another step only where the two are within bf16 noise (a near tie); a
# wrong argmax lands far below the max.
POOL_ROUTE_RTOL = None


def mean_max_pool(x):
    """cat(mean over time, max over time) -- cmu-mosei/run.py:318 (padded rows included)."""
    if POOL_ROUTE:
        idx = POOL_ROUTE.pop(0).to(x.device).long()
        mx = x.gather(1, idx.unsqueeze(1)).squeeze(1)
        if POOL_ROUTE_RTOL is not None:
            with torch.no_grad():
                gap = x.max(dim=1).values - mx
                lim = POOL_ROUTE_RTOL * x.abs().amax(dim=1)
                bad = gap > lim
                assert not bool(bad.any()), ('routed max-pool: %d of %d replayed steps fall below the column max by '
                                             'more than %.3g of its scale (worst gap %.3g)'
                                             % (int(bad.sum()), bad.numel(), POOL_ROUTE_RTOL, float((gap - lim).max())))
    else:
        mx, idx = x.max(dim=1)
    POOL_SEEN.append(idx.detach().clone())
    return torch.cat([x.mean(dim=1), mx], dim=1)


def bilinear_transfer(this, last, trans):
    """y[b,n] = sum_{p,m} this[b,p] last[b,m] trans[p,m,n], one row at a time as the reference
    does (cmu-mosei/run.py:332-337, Ren-MME/run.py:285-290): ``(last[i] @ trans)`` then
    ``this[i] @ .``."""
    rows = []
    for i in range(this.shape[0]):
        t = torch.matmul(last[i], trans)
        rows.append(torch.matmul(this[i], t).unsqueeze(0))
    return torch.cat(rows, dim=0)


def circle_loss(y_pred, y_true):
    """Per-row multi-label circle loss, cmu-mosei/run.py:342-351 (realformer.py:289-298,
    Ren-MME/run.py:295-303 before its .mean())."""
    y_true = y_true.to(y_pred.dtype) if y_true.dtype.is_floating_point else y_true
    y = (1 - 2 * y_true) * y_pred
    neg = y - y_true * CIRCLE_BIG
    pos = y - (1 - y_true) * CIRCLE_BIG
    z = torch.zeros_like(y[..., :1], dtype=torch.float)
    return torch.logsumexp(torch.cat([neg, z], -1), -1) + torch.logsumexp(torch.cat([pos, z], -1), -1)


def rdrop_kl(logits):
    """Symmetric R-Drop KL between duplicate rows, Ren-MME/run.py:332-334:
    0.5*(KL(sig(q)||logsig(p)) + KL(sig(p)||logsig(q))), reduction batchmean."""
    f = torch.nn.functional
    p, q = logits[::2], logits[1::2]
    k0 = f.kl_div(f.logsigmoid(p), torch.sigmoid(q), reduction='batchmean')
    k1 = f.kl_div(f.logsigmoid(q), torch.sigmoid(p), reduction='batchmean')
    return (k0 + k1) / 2


# ----------------------------------------------------------------------------- optimizer step

def clip_grad_norm(grads, max_norm):
    """torch.nn.utils.clip_grad_norm_ semantics (cmu-mosei/run.py:368): grads that are None
    are skipped; total = ||concat||_2; coef = min(max_norm/(total+1e-6), 1)."""
    gs = [g for g in grads if g is not None]
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g, 2) for g in gs]), 2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in gs:
        g.mul_(coef)
    return total


class AdamState:
    """torch.optim.AdamW / Adam (single-tensor, non-amsgrad) restated.  AdamW defaults as used at
    cmu-mosei/run.py:398 (lr given, betas (0.9,0.999), eps 1e-8, weight_decay 0.01); Adam at
    others/realformer.py:342 (weight_decay 0, no decoupled decay).  Parameters whose grad is None
    are skipped entirely (no decay, no step count) as torch does."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 decoupled=True):
        self.params = list(params)
        self.lr, self.betas, self.eps, self.wd, self.decoupled = lr, betas, eps, weight_decay, decoupled
        self.state = {}

    @torch.no_grad()
    def step(self):
        b1, b2 = self.betas
        for i, p in enumerate(self.params):
            g = p.grad
            if g is None:
                continue
            st = self.state.setdefault(i, {'t': 0, 'm': torch.zeros_like(p), 'v': torch.zeros_like(p)})
            st['t'] += 1
            t = st['t']
            if self.decoupled:
                p.mul_(1 - self.lr * self.wd)
            elif self.wd != 0:
                g = g.add(p, alpha=self.wd)
            st['m'].lerp_(g, 1 - b1)
            st['v'].mul_(b2).addcmul_(g, g, value=1 - b2)
            bc1 = 1 - b1 ** t
            bc2 = 1 - b2 ** t
            denom = (st['v'].sqrt() / math.sqrt(bc2)).add_(self.eps)
            p.addcdiv_(st['m'], denom, value=-(self.lr / bc1))
