"""Standalone execution of single reference sub-modules on libmep_hip (not the fused step).

``Attention_Block.forward(q, k, v, mask, scores)`` (cmu-mosei/run.py:258-262) and
``Unify_Dimension.forward`` (run.py:213-214) called directly by user code run here: the same
kernels as the fused plan, with one descriptor per launch built per call.  The model-level
forward (Concat_Trans / Base_model) never comes through this module.
"""
import ctypes

import torch

from . import _lib
from ._lib import (AttnBwdDesc, AttnDesc, ColsumDesc, DescArray, EpiBwdDesc, EpiDesc, GemmDesc, Rows,
                   launch)
from .trimodal import cdiv, crows, make_wgrad


def _c(t):
    """contiguous fp32 with a 16-byte aligned base (the kernels read rows with 16-byte loads)"""
    t = t.contiguous().float()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _wgrad(items, dev):
    ws, arr, tmax, rmax = make_wgrad(items, dev)
    launch('mep_wgrad', arr, tmax)
    launch('mep_wgrad_reduce', arr, rmax)
    return ws, arr


def _mask_of(mask, q, k):
    """The reference's mask forms (cmu-mosei/run.py:247-252) -> (fp32 mask tensor, 3-D?):
    None -> an all-ones [B, Tk] key mask (the reference subtracts nothing; s - 1e8 * (1 - 1) is
    s - 0 = s, bit for bit), [B, Tk] -> the key mask of the fused kernels, [B, Tq, Tk] -> the
    general kernels (mep_attn_general_*)."""
    B, Tq, Tk = q.shape[0], q.shape[1], k.shape[1]
    if mask is None:
        return torch.ones(B, Tk, dtype=torch.float32, device=q.device), False
    if mask.dim() == 2 and tuple(mask.shape) == (B, Tk):
        return _c(mask), False
    if mask.dim() == 3 and tuple(mask.shape) == (B, Tq, Tk):
        return _c(mask), True
    raise ValueError('mask must be None, [batch, kv_len] or [batch, q_len, kv_len]; got %s' % (tuple(mask.shape),))


def _gen_desc(ad, H, D, Tq, Tk):
    """mep_attn_gen_desc of a [B, Tq, Tk] mask: scale = float32(np.sqrt(hd)), the divisor the
    reference's q @ k^T / np.sqrt(k.size(-1)) uses"""
    import numpy as np
    hd = D // H
    ad.mask_sB = Tq * Tk
    return _lib.AttnGenDesc(f=ad, mask_sQ=Tk, hd=hd, scale=float(np.float32(np.sqrt(hd))))


def _advance_seed(seed):
    _lib.call('mep_seed_advance', ctypes.c_void_p(seed.data_ptr()))


class _BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, H, drop_p, seed, q, k, v, mask, s_prev, c, wp, wm, lnw, lnb):
        q, k, v = _c(q), _c(k), _c(v)
        mask, general = _mask_of(mask, q, k)
        B, Tq, D = q.shape
        Tk = k.shape[1]
        dev = q.device
        same_kv = k.data_ptr() == v.data_ptr()
        f = dict(dtype=torch.float32, device=dev)
        X, XP, Z, out = (torch.empty(B, Tq, D, **f) for _ in range(4))
        S = torch.empty(B, H, Tq, Tk, **f)
        astat = torch.empty(3 * B * H * Tq, **f)   # (max, 1/sum) per row, then S_prev means (mep.h)
        estat = torch.empty(B * Tq, 2, **f)
        sp = _c(s_prev) if s_prev is not None else None
        ad = AttnDesc(q=crows(q, Tq, D), k=crows(k, Tk, D), v=crows(v, Tk, D), x=crows(X, Tq, D),
                      mask=mask.data_ptr(), mask_sB=Tk, s_prev=sp.data_ptr() if sp is not None else 0,
                      c=c.data_ptr(), s_out=S.data_ptr(), stats=astat.data_ptr(), B=B, H=H, Tq=Tq, Tk=Tk)
        wp, wm = _c(wp), _c(wm)
        # training-mode dropout (Ren-MME DROP = 0.1, run.py:173, 209, 213): the epilogue's two
        # sites on the counter-hash masks of the block's seed, advanced per forward like a fresh
        # nn.Dropout draw; the forward records the keep bits the backward reads
        bits = torch.zeros(cdiv(B * Tq, 16), 2, 64, dtype=torch.int32, device=dev) if drop_p > 0.0 else None
        if bits is not None:
            _advance_seed(seed)
        ed = EpiDesc(q=crows(q, Tq, D), x=crows(X, Tq, D), xp=crows(XP, Tq, D), z=crows(Z, Tq, D),
                     out=crows(out, Tq, D), wp=wp.data_ptr(), wm=wm.data_ptr(), ln_w=lnw.data_ptr(),
                     ln_b=lnb.data_ptr(), stats=estat.data_ptr(), seed=seed.data_ptr() if bits is not None else 0,
                     ntok=B * Tq, D=D, drop_p=drop_p if bits is not None else 0.0, drop_stream=0,
                     drop_bits=bits.data_ptr() if bits is not None else 0)
        e_arr = DescArray(EpiDesc, [ed], dev)
        if general:
            gd = _gen_desc(ad, H, D, Tq, Tk)
            _lib.call('mep_attn_general_fwd', DescArray(_lib.AttnGenDesc, [gd], dev).ptr, 1, B * H)
        else:
            gd = None
            geo = _lib.attn_geometry([ad])
            launch('mep_attn_fwd', DescArray(AttnDesc, [ad], dev), geo[0], threads=geo[2])
        launch('mep_block_epi_fwd', e_arr, _lib.epi_grid(B * Tq, 1), threads=D)
        ctx.save_for_backward(q, k, v, mask, X, XP, Z, S, astat, estat, c, wp, wm, lnw, lnb)
        ctx.sp, ctx.bits, ctx.seed = sp, bits, seed
        ctx.meta = (B, Tq, Tk, D, H, same_kv)
        ctx.descs = (ad, ed, gd)
        return out, S

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout, dS):
        (q, k, v, mask, X, XP, Z, S, astat, estat, c, wp, wm, lnw, lnb) = ctx.saved_tensors
        B, Tq, Tk, D, H, same_kv = ctx.meta
        ad, ed, gd = ctx.descs
        dev = q.device
        f = dict(dtype=torch.float32, device=dev)
        dout = _c(dout) if dout is not None else torch.zeros(B, Tq, D, **f)
        dS = _c(dS) if dS is not None else None
        dZ, dXP, dX, dQ = (torch.empty(B, Tq, D, **f) for _ in range(4))
        dK = torch.empty(B, Tk, D, **f)
        dV = dK if same_kv else torch.empty(B, Tk, D, **f)
        ln_part = torch.empty(cdiv(B * Tq, 16), 2, D, **f)
        has_prev = ctx.sp is not None
        dSp = torch.empty(B, H, Tq, Tk, **f) if has_prev else None
        n_dc = B * H if gd is not None else _lib.attn_dc_slots(B, H, Tk)
        dc_part = torch.empty(n_dc, **f) if has_prev else None
        eb = EpiBwdDesc(f=ed, dout=crows(dout, Tq, D), dout2=Rows(), dz=crows(dZ, Tq, D), dxp=crows(dXP, Tq, D),
                        dx=crows(dX, Tq, D), dq=crows(dQ, Tq, D), ln_partial=ln_part.data_ptr(), dq_accumulate=0)
        launch('mep_block_epi_bwd', DescArray(EpiBwdDesc, [eb], dev), _lib.epi_grid(B * Tq, 1), threads=D)
        outs = dict(dx=crows(dX, Tq, D), dq=crows(dQ, Tq, D), dk=crows(dK, Tk, D), dv=crows(dV, Tk, D),
                    ds_next=dS.data_ptr() if dS is not None else 0, ds_prev=dSp.data_ptr() if has_prev else 0,
                    dc_partial=dc_part.data_ptr() if has_prev else 0)
        if gd is not None:
            gb = _lib.AttnGenBwdDesc(g=gd, **outs)
            _lib.call('mep_attn_general_bwd', DescArray(_lib.AttnGenBwdDesc, [gb], dev).ptr, 1, B * H, gd.hd)
        else:
            ab = AttnBwdDesc(f=ad, **outs)
            geo = _lib.attn_geometry([ad])
            launch('mep_attn_bwd', DescArray(AttnBwdDesc, [ab], dev), geo[1], threads=_lib.attn_bwd_flags([ab]))
        gwp, gwm = torch.empty_like(wp), torch.empty_like(wm)
        glw, glb, gc = torch.empty_like(lnw), torch.empty_like(lnb), torch.empty_like(c)
        n = B * Tq
        keep = _wgrad([(crows(dXP, Tq, D), D, n, [(crows(X, Tq, D), D, gwp.data_ptr(), D)]),
                       (crows(dZ, Tq, D), D, n, [(crows(q, Tq, D), D, gwm.data_ptr(), 2 * D),
                                                 (crows(XP, Tq, D), D, gwm.data_ptr() + 4 * D, 2 * D)])], dev)
        cs = [ColsumDesc(partial=ln_part.data_ptr(), out=glw.data_ptr(), n_rows=ln_part.shape[0], n_cols=D,
                         ld=2 * D, accumulate=0),
              ColsumDesc(partial=ln_part.data_ptr() + 4 * D, out=glb.data_ptr(), n_rows=ln_part.shape[0],
                         n_cols=D, ld=2 * D, accumulate=0)]
        if has_prev:
            cs.append(ColsumDesc(partial=dc_part.data_ptr(), out=gc.data_ptr(), n_rows=dc_part.numel(), n_cols=1,
                                 ld=1, accumulate=0))
        launch('mep_colsum', DescArray(ColsumDesc, cs, dev), cdiv(D, 32))
        del keep
        return (None, None, None, dQ, dK, None if same_kv else dV, None, dSp, gc if has_prev else None,
                gwp, gwm, glw, glb)


def block_seed(block, device):
    """The standalone block's dropout seed state (device uint64 {seed, row0 = 0}, the plans'
    layout): drawn from torch's generator on first use, advanced on the device by every
    training-mode forward (a fresh mask per call, as nn.Dropout draws)"""
    s = getattr(block, '_mep_seed', None)
    if s is None or s.device != torch.device(device):
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        s = torch.tensor([seed, 0], dtype=torch.int64, device=device)
        block._mep_seed = s
    return s


def block_forward(block, q, k, v, mask, scores, norm, drop_p=0.0):
    """cmu-mosei / Ren-MME Attention_Block.forward(q, k, v, mask, scores=None): every mask form the
    reference accepts (None, [B, Tk], [B, Tq, Tk]) and, in training mode, the block's dropout."""
    from ._autograd import require_cuda
    require_cuda(q, k, v, mask)
    p = float(drop_p) if block.training else 0.0
    seed = block_seed(block, q.device) if p > 0.0 else torch.zeros(2, dtype=torch.int64, device=q.device)
    return _BlockFn.apply(block.n_heads, p, seed, q, k, v, mask, scores, block.c, block.proj.weight,
                          block.minus.weight, norm.weight, norm.bias)


class _UnifyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        x = _c(x)
        lead = x.shape[:-1]
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K)
        n = x2.shape[0]
        y = torch.empty(n, N, dtype=torch.float32, device=x.device)
        d = GemmDesc(x=crows(x2, n, K), y=crows(y, n, N), w=w.data_ptr(), bias=0, table=0, ntok=n, N=N, K=K, ldw=K,
                     w_nt=1, accumulate=0, relu=0, alpha=1.0)
        launch('mep_gemm', DescArray(GemmDesc, [d], x.device), cdiv(n, 64))
        ctx.save_for_backward(x2, w)
        ctx.x_shape = x.shape
        return y.reshape(*lead, N)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        n, K = x2.shape
        N = w.shape[0]
        gy = _c(gy).reshape(n, N)
        gw = torch.empty_like(w)
        keep = _wgrad([(crows(gy, n, N), N, n, [(crows(x2, n, K), K, gw.data_ptr(), K)])], x2.device)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty(n, K, dtype=torch.float32, device=x2.device)
            d = GemmDesc(x=crows(gy, n, N), y=crows(gx, n, K), w=w.data_ptr(), bias=0, table=0, ntok=n, N=K, K=N,
                         ldw=K, w_nt=0, accumulate=0, relu=0, alpha=1.0)
            launch('mep_gemm', DescArray(GemmDesc, [d], x2.device), cdiv(n, 64))
            gx = gx.reshape(ctx.x_shape)
        del keep
        return gx, gw


def linear_nobias(x, w):
    from ._autograd import require_cuda
    require_cuda(x)
    return _UnifyFn.apply(x, w)


def unify_forward(mod, l, v, a):
    return (linear_nobias(l, mod.linguistic.weight), linear_nobias(v, mod.visual.weight),
            linear_nobias(a, mod.acoustic.weight))


class _LayerNormFn(torch.autograd.Function):
    """Row LayerNorm on libmep_hip (Ren-MME's shared unify norm1, Ren-MME/run.py:164-166)."""

    @staticmethod
    def forward(ctx, x, w, b):
        shape = x.shape
        D = shape[-1]
        x2 = _c(x).reshape(-1, D)
        ntok = x2.shape[0]
        dev = x.device
        y = torch.empty_like(x2)
        stats = torch.empty(ntok, 2, dtype=torch.float32, device=dev)
        d = _lib.LnDesc(x=crows(x2, 1, D), y=crows(y, 1, D), dy=Rows(), dx=Rows(), w=w.data_ptr(), b=b.data_ptr(),
                        stats=stats.data_ptr(), partial=0, ntok=ntok, D=D, dx_accumulate=0)
        launch('mep_layernorm_fwd', DescArray(_lib.LnDesc, [d], dev), cdiv(ntok, 4))
        ctx.save_for_backward(x2, w, stats)
        ctx.shape = shape
        return y.reshape(shape)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gy):
        x2, w, stats = ctx.saved_tensors
        ntok, D = x2.shape
        dev = x2.device
        gy = _c(gy).reshape(-1, D)
        dx = torch.empty_like(x2)
        tiles = cdiv(ntok, 64)
        partial = torch.empty(tiles, 2, D, dtype=torch.float32, device=dev)
        d = _lib.LnDesc(x=crows(x2, 1, D), y=Rows(), dy=crows(gy, 1, D), dx=crows(dx, 1, D), w=w.data_ptr(), b=0,
                        stats=stats.data_ptr(), partial=partial.data_ptr(), ntok=ntok, D=D, dx_accumulate=0)
        launch('mep_layernorm_bwd', DescArray(_lib.LnDesc, [d], dev), tiles)
        gw = torch.empty(D, dtype=torch.float32, device=dev)
        gb = torch.empty(D, dtype=torch.float32, device=dev)
        cs = [ColsumDesc(partial=partial.data_ptr(), out=gw.data_ptr(), n_rows=tiles, n_cols=D, ld=2 * D,
                         accumulate=0),
              ColsumDesc(partial=partial.data_ptr() + 4 * D, out=gb.data_ptr(), n_rows=tiles, n_cols=D, ld=2 * D,
                         accumulate=0)]
        launch('mep_colsum', DescArray(ColsumDesc, cs, dev), cdiv(D, 32))
        return dx.reshape(ctx.shape), gw, gb


def layer_norm(x, norm):
    from ._autograd import require_cuda
    require_cuda(x)
    assert norm.weight.shape[0] <= 256, 'mep_layernorm supports D <= 256'
    return _LayerNormFn.apply(x, norm.weight, norm.bias)


def unify_norm_forward(mod, l, v, a):
    """Ren-MME Unify_Dimension.forward (Ren-MME/run.py:167-168): shared norm1 after each projection."""
    return tuple(layer_norm(y, mod.norm1) for y in unify_forward(mod, l, v, a))


class _RFBlockFn(torch.autograd.Function):
    """realformer Attention_Block.forward (others/realformer.py:182-209) on libmep_hip:
    Q/K/V projections (mep_gemm), residual attention core, fused RealFormer epilogue."""

    @staticmethod
    def forward(ctx, H, q, k, v, mask, s_prev, wq, wk, wv, wp, n1w, n1b, n2w, n2b, w1, b1, w2, b2, a, b, c):
        q, k, v = _c(q), _c(k), _c(v)
        mask, general = _mask_of(mask, q, k)
        B, Tq, D = q.shape
        Tk = k.shape[1]
        FD = w1.shape[0]
        dev = q.device
        f = dict(dtype=torch.float32, device=dev)
        QP, X, XP, Hh, F, out = (torch.empty(B, Tq, D, **f) for _ in range(6))
        KV = torch.empty(B, Tk, 2 * D, **f)
        F1 = torch.empty(B, Tq, FD, **f)
        S = torch.empty(B, H, Tq, Tk, **f)
        astat = torch.empty(3 * B * H * Tq, **f)   # (max, 1/sum) per row, then S_prev means (mep.h)
        estat = torch.empty(B * Tq, 4, **f)
        sp = _c(s_prev) if s_prev is not None else None
        kv = lambda t, which: _lib.Rows(ptr=t.data_ptr() + 4 * which * D, sB=Tk * 2 * D, sT=2 * D, T=Tk)  # noqa: E731
        g = dict(bias=0, table=0, accumulate=0, relu=0, alpha=1.0, w_nt=1, K=D, ldw=D, N=D)
        gd = [GemmDesc(x=crows(q, Tq, D), y=crows(QP, Tq, D), w=wq.data_ptr(), ntok=B * Tq, **g),
              GemmDesc(x=crows(k, Tk, D), y=kv(KV, 0), w=wk.data_ptr(), ntok=B * Tk, **g),
              GemmDesc(x=crows(v, Tk, D), y=kv(KV, 1), w=wv.data_ptr(), ntok=B * Tk, **g)]
        launch('mep_gemm', DescArray(GemmDesc, gd, dev), cdiv(B * max(Tq, Tk), 64))
        ad = AttnDesc(q=crows(QP, Tq, D), k=kv(KV, 0), v=kv(KV, 1), x=crows(X, Tq, D), mask=mask.data_ptr(),
                      mask_sB=Tk, s_prev=sp.data_ptr() if sp is not None else 0, c=c.data_ptr(), s_out=S.data_ptr(),
                      stats=astat.data_ptr(), B=B, H=H, Tq=Tq, Tk=Tk)
        ed = _lib.RfEpiDesc(q=crows(q, Tq, D), x=crows(X, Tq, D), xp=crows(XP, Tq, D), h=crows(Hh, Tq, D),
                            f1=crows(F1, Tq, FD), f=crows(F, Tq, D), out=crows(out, Tq, D), wp=wp.data_ptr(),
                            w1=w1.data_ptr(), b1=b1.data_ptr(), w2=w2.data_ptr(), b2=b2.data_ptr(),
                            ln1_w=n1w.data_ptr(), ln1_b=n1b.data_ptr(), ln2_w=n2w.data_ptr(), ln2_b=n2b.data_ptr(),
                            a=a.data_ptr(), b=b.data_ptr(), stats=estat.data_ptr(), ntok=B * Tq, D=D, FD=FD)
        if general:
            gd = _gen_desc(ad, H, D, Tq, Tk)
            _lib.call('mep_attn_general_fwd', DescArray(_lib.AttnGenDesc, [gd], dev).ptr, 1, B * H)
        else:
            gd = None
            geo = _lib.attn_geometry([ad])
            launch('mep_attn_fwd', DescArray(AttnDesc, [ad], dev), geo[0], threads=geo[2])
        rfw = _lib.RFW
        ctx.wbuf = None
        if rfw:   # the epilogue's Linears on mep_wsplit parts (wave-tiled kernels, csrc/rfw.hip)
            arena = _lib.PartsArena()
            off = arena.add_epi(D, FD, wp.data_ptr(), w1.data_ptr(), w2.data_ptr())
            ctx.wbuf, wsd, units = arena.build(dev)
            launch('mep_wsplit', wsd, units)
            ed.wparts = ctx.wbuf.data_ptr() + off
        launch('mep_rfw_epi_fwd' if rfw else 'mep_rf_epi_fwd', DescArray(_lib.RfEpiDesc, [ed], dev),
               cdiv(B * Tq, _lib.rf_epi_rows(D, rfw)), extra=(D, FD))
        ctx.rfw = rfw
        ctx.save_for_backward(q, k, v, mask, QP, KV, X, XP, Hh, F1, F, S, astat, estat,
                              wq, wk, wv, wp, n1w, n1b, n2w, n2b, w1, b1, w2, b2, a, b, c)
        ctx.sp = sp
        ctx.meta = (B, Tq, Tk, D, H, FD)
        ctx.descs = (ad, ed, gd)
        return out, S

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout, dS):
        (q, k, v, mask, QP, KV, X, XP, Hh, F1, F, S, astat, estat,
         wq, wk, wv, wp, n1w, n1b, n2w, n2b, w1, b1, w2, b2, a, b, c) = ctx.saved_tensors
        B, Tq, Tk, D, H, FD = ctx.meta
        ad, ed, gd = ctx.descs
        dev = q.device
        f = dict(dtype=torch.float32, device=dev)
        dout = _c(dout) if dout is not None else torch.zeros(B, Tq, D, **f)
        dS = _c(dS) if dS is not None else None
        dF, dXP, dX, dQin = (torch.empty(B, Tq, D, **f) for _ in range(4))
        dQP = torch.zeros(B, Tq, D, **f)
        dF1 = torch.empty(B, Tq, FD, **f)
        dKV2 = torch.empty(B, Tk, 2 * D, **f)
        dk_in, dv_in = torch.empty(B, Tk, D, **f), torch.empty(B, Tk, D, **f)
        nt = cdiv(B * Tq, _lib.rf_bwd_rows(ctx.rfw))
        stride = _lib.rf_partial_stride(D, FD)
        part = torch.empty(nt, stride, **f)
        has_prev = ctx.sp is not None
        dSp = torch.empty(B, H, Tq, Tk, **f) if has_prev else None
        dc_part = torch.empty(B * H if gd is not None else _lib.attn_dc_slots(B, H, Tk), **f) if has_prev else None
        kv = lambda t, which: _lib.Rows(ptr=t.data_ptr() + 4 * which * D, sB=Tk * 2 * D, sT=2 * D, T=Tk)  # noqa: E731
        eb = _lib.RfEpiBwdDesc(f=ed, dout=crows(dout, Tq, D), dout2=Rows(), df=crows(dF, Tq, D),
                               df1=crows(dF1, Tq, FD), dxp=crows(dXP, Tq, D), dx=crows(dX, Tq, D),
                               dq=crows(dQin, Tq, D), partial=part.data_ptr(), dq_accumulate=0)
        outs = dict(dx=crows(dX, Tq, D), dq=crows(dQP, Tq, D), dk=kv(dKV2, 0), dv=kv(dKV2, 1),
                    ds_next=dS.data_ptr() if dS is not None else 0, ds_prev=dSp.data_ptr() if has_prev else 0,
                    dc_partial=dc_part.data_ptr() if has_prev else 0)
        launch('mep_rfw_epi_bwd' if ctx.rfw else 'mep_rf_epi_bwd', DescArray(_lib.RfEpiBwdDesc, [eb], dev), nt,
               extra=(D, FD))
        if gd is not None:
            gb = _lib.AttnGenBwdDesc(g=gd, **outs)
            _lib.call('mep_attn_general_bwd', DescArray(_lib.AttnGenBwdDesc, [gb], dev).ptr, 1, B * H, gd.hd)
        else:
            ab = AttnBwdDesc(f=ad, **outs)
            geo = _lib.attn_geometry([ad])
            launch('mep_attn_bwd', DescArray(AttnBwdDesc, [ab], dev), geo[1], threads=_lib.attn_bwd_flags([ab]))
        g = dict(bias=0, table=0, relu=0, alpha=1.0, w_nt=0, K=D, ldw=D, N=D)
        gd = [GemmDesc(x=crows(dQP, Tq, D), y=crows(dQin, Tq, D), w=wq.data_ptr(), ntok=B * Tq, accumulate=1, **g),
              GemmDesc(x=kv(dKV2, 0), y=crows(dk_in, Tk, D), w=wk.data_ptr(), ntok=B * Tk, accumulate=0, **g),
              GemmDesc(x=kv(dKV2, 1), y=crows(dv_in, Tk, D), w=wv.data_ptr(), ntok=B * Tk, accumulate=0, **g)]
        launch('mep_gemm', DescArray(GemmDesc, gd, dev), cdiv(B * max(Tq, Tk), 64))
        grads = {name: torch.empty_like(t) for name, t in (('wq', wq), ('wk', wk), ('wv', wv), ('wp', wp),
                                                           ('n1w', n1w), ('n1b', n1b), ('n2w', n2w), ('n2b', n2b),
                                                           ('w1', w1), ('b1', b1), ('w2', w2), ('b2', b2),
                                                           ('a', a), ('b', b), ('c', c))}
        nq, nk = B * Tq, B * Tk
        keep = _wgrad([(crows(dQP, Tq, D), D, nq, [(crows(q, Tq, D), D, grads['wq'].data_ptr(), D)]),
                       (kv(dKV2, 0), D, nk, [(crows(k, Tk, D), D, grads['wk'].data_ptr(), D)]),
                       (kv(dKV2, 1), D, nk, [(crows(v, Tk, D), D, grads['wv'].data_ptr(), D)]),
                       (crows(dXP, Tq, D), D, nq, [(crows(X, Tq, D), D, grads['wp'].data_ptr(), D)]),
                       (crows(Hh, Tq, D), D, nq, [(crows(dF1, Tq, FD), FD, grads['w1'].data_ptr(), D)], 1),
                       (crows(dF, Tq, D), D, nq, [(crows(F1, Tq, FD), FD, grads['w2'].data_ptr(), FD)])], dev)
        cs = []
        for k_, (name, n) in enumerate((('n2w', D), ('n2b', D), ('n1w', D), ('n1b', D), ('b2', D))):
            cs.append(ColsumDesc(partial=part.data_ptr() + 4 * k_ * D, out=grads[name].data_ptr(), n_rows=nt,
                                 n_cols=n, ld=stride, accumulate=0))
        for name, off, n in (('b1', 5 * D, FD), ('a', 5 * D + FD, 1), ('b', 5 * D + FD + 1, 1)):
            cs.append(ColsumDesc(partial=part.data_ptr() + 4 * off, out=grads[name].data_ptr(), n_rows=nt, n_cols=n,
                                 ld=stride, accumulate=0))
        if has_prev:
            cs.append(ColsumDesc(partial=dc_part.data_ptr(), out=grads['c'].data_ptr(), n_rows=dc_part.numel(),
                                 n_cols=1, ld=1, accumulate=0))
        launch('mep_colsum', DescArray(ColsumDesc, cs, dev), cdiv(max(D, FD), 32))
        del keep
        return (None, dQin, dk_in, dv_in, None, dSp, grads['wq'], grads['wk'], grads['wv'], grads['wp'],
                grads['n1w'], grads['n1b'], grads['n2w'], grads['n2b'], grads['w1'], grads['b1'], grads['w2'],
                grads['b2'], grads['a'], grads['b'], grads['c'] if has_prev else None)


def rf_block_forward(block, q, k, v, mask, scores):
    from ._autograd import require_cuda
    require_cuda(q, k, v, mask)
    if block.training and block.drop.p > 0.0:
        raise NotImplementedError('realformer dropout: the reference runs DROP = 0 (others/realformer.py:37)')
    ffn0, ffn2 = block.ffn[0], block.ffn[2]
    return _RFBlockFn.apply(block.n_heads, q, k, v, mask, scores, block.w_qkv[0].weight, block.w_qkv[1].weight,
                            block.w_qkv[2].weight, block.proj.weight, block.norm1.weight, block.norm1.bias,
                            block.norm2.weight, block.norm2.bias, ffn0.weight, ffn0.bias, ffn2.weight, ffn2.bias,
                            block.a, block.b, block.c)


# ---------------------------------------------------------------- standalone encoders
# Multi_ATTN.forward (cmu-mosei/run.py:272-319, Ren-MME/run.py:224-277) and Multi_class.forward
# (others/realformer.py:223-264) as their own entries: the unify projection and every block run
# on the HIP kernels above (one grouped launch sequence each, with its own backward); the
# concatenation of the chain outputs, the mean / max pool over time and the classifier (or
# FC + LayerNorm + ReLU) are PyTorch-ROCm ops.  The training hot path never comes here:
# Concat_Trans / Base_model / State_Transfer run both encoders, pool and head as one plan.
def encoder_features(mod, feats, masks, every_layer):
    """The nine chains of an encoder over unified features: feats / masks {'l','v','a'} ->
    [B, T_l + T_a + T_v, 3 * D * (n_layers if every_layer else 1)], chain outputs concatenated
    per query modality in chain order (every layer's output for cmu-mosei / Ren-MME,
    cmu-mosei/run.py:279-313; the last layer's for realformer, realformer.py:231-259) and the
    modalities along time in the order l, a, v (cmu-mosei/run.py:317)."""
    from .trimodal import CHAINS, TIME_ORDER
    nl = mod.n_layers
    rows = {'l': [], 'v': [], 'a': []}
    for j, (qm, km) in enumerate(CHAINS):
        x, s = feats[qm], None
        for i in range(nl):
            x, s = mod.multimodal_blocks[nl * j + i](x, feats[km], feats[km], masks[km], s)
            if every_layer:
                rows[qm].append(x)
        if not every_layer:
            rows[qm].append(x)
    return torch.cat([torch.cat(rows[m], dim=2) for m in TIME_ORDER], dim=1)


def mean_max_pool(x):
    """torch.cat([mean(x, 1), max(x, 1)[0]], 1) (cmu-mosei/run.py:318; padded steps included), with
    the max's gradient routed to the FIRST maximal step -- the reference's (CPU) tie-break, which
    the fused pool kernel follows too.  Ties are common: every padded step of a row has zero
    features and the same block output."""
    mx = x.detach().amax(1, keepdim=True)
    steps = torch.arange(x.shape[1], device=x.device).view(1, -1, 1)
    first = torch.where(x.detach() == mx, steps, x.shape[1]).amin(1, keepdim=True)
    return torch.cat([x.mean(1), x.gather(1, first).squeeze(1)], dim=1)


def multi_attn_forward(mod, l, v, a, l_mask, v_mask, a_mask):
    """cmu-mosei / Ren-MME Multi_ATTN.forward -> classifier logits."""
    from ._autograd import require_cuda
    require_cuda(l, v, a, l_mask, v_mask, a_mask)
    u = dict(zip('lva', mod.unify_dimension(l, v, a)))
    x = encoder_features(mod, u, {'l': l_mask, 'v': v_mask, 'a': a_mask}, every_layer=True)
    return mod.classifier(mean_max_pool(x))


def multi_class_forward(mod, l, v, a, l_mask, v_mask, a_mask):
    """realformer Multi_class.forward -> [B, D] (Conv1d unify + position embedding, nine chains,
    pool, FC, LayerNorm, ReLU, dropout p = 0)."""
    from ._autograd import require_cuda
    require_cuda(l, v, a, l_mask, v_mask, a_mask)
    ul, uv, ua = mod.unify_dimension(l, v, a)
    u = {'l': ul + mod.linguistic_position(ul), 'v': uv + mod.visual_position(uv),
         'a': ua + mod.acoustic_position(ua)}
    x = encoder_features(mod, u, {'l': l_mask, 'v': v_mask, 'a': a_mask}, every_layer=False)
    x = torch.relu(mod.normalization(mod.fully_connected(mean_max_pool(x))))
    return mod.drop(x)
