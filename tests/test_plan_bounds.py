"""Host-logic check of the execution plans (CPU, no GPU): every device range any descriptor of a
plan names -- operand rows, weights, workspaces, partials -- lies inside one buffer the plan (or
its flat parameter store) owns.  A descriptor that points past a buffer would be a GPU memory
fault; this catches it before any kernel runs.  Plans are built on CPU tensors (descriptor
building only; nothing is launched)."""
import ctypes

import pytest
import torch

from mep_amd import _lib
from mep_amd._lib import (AttnBwdDesc, AttnDesc, ColsumDesc, EpiBwdDesc, EpiDesc, GemmDesc, HeadDesc, LnDesc,
                          PoolDesc, SumDesc, WgradDesc)
from mep_amd.trimodal import cdiv

F = 4


def _tensors(obj, out, depth=0):
    if torch.is_tensor(obj):
        out.append(obj)
    elif isinstance(obj, dict):
        for v in obj.values():
            _tensors(v, out, depth + 1)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _tensors(v, out, depth + 1)
    elif depth < 2 and hasattr(obj, '__dict__') and not isinstance(obj, type):
        for v in vars(obj).values():
            _tensors(v, out, depth + 1)
    return out


class Checker:
    def __init__(self, plan):
        ts = _tensors(plan, [])
        fl = plan.flat
        ts += [fl.buf, fl.grad]
        # whole storages (a view's data_ptr plus its storage's size would run past the storage)
        self.allocs = sorted({(t.untyped_storage().data_ptr(), t.untyped_storage().nbytes(), t.element_size())
                              for t in ts if t.numel()})
        self.n = 0

    def inside(self, label, ptr, nbytes):
        if ptr == 0 or nbytes <= 0:
            return
        self.n += 1
        for base, size, _ in self.allocs:
            if base <= ptr and ptr + nbytes <= base + size:
                return
        raise AssertionError('%s: [%#x, +%d) is outside every plan buffer' % (label, ptr, nbytes))

    def elsize(self, ptr):
        """bytes per element of the buffer a row view points into (bf16 activations on the bf16
        path, include/mep.h MEP_PREC_BF16)"""
        for base, size, es in self.allocs:
            if base <= ptr < base + size:
                return es
        return F

    def rows(self, label, r, ntok, cols, es=None):
        if r.ptr == 0 or ntok == 0:
            return
        assert r.T > 0, label
        last = (ntok - 1) // r.T * r.sB + (ntok - 1) % r.T * r.sT
        self.inside(label, r.ptr, (last + cols) * (es or self.elsize(r.ptr)))


def _decode(arr):
    if arr is None or arr.n == 0:
        return []
    raw = bytes(arr.dev.cpu().numpy().tobytes())
    sz = ctypes.sizeof(arr.struct)
    return [arr.struct.from_buffer_copy(raw[i * sz:(i + 1) * sz]) for i in range(arr.n)]


def _gemm(c, d, parts=False):
    """parts: the weight is a mep_wsplit parts image (wave-tiled realformer path: mep_wgemm reads
    W' [N][K] as three bf16 parts with rows padded to 32), not the fp32 parameter"""
    c.rows('gemm.x', d.x, d.ntok, d.K)
    c.rows('gemm.y', d.y, d.ntok, d.N)
    if parts:
        c.inside('gemm.wparts', d.w, _lib.wsplit_bytes(cdiv(d.N, 32) * 32, d.K))
    else:
        c.inside('gemm.w', d.w, ((d.N - 1) * d.ldw + d.K if d.w_nt else (d.K - 1) * d.ldw + d.N) * F)
    c.inside('gemm.bias', d.bias, d.N * F)
    c.inside('gemm.table', d.table, d.y.T * d.N * F)


def _wgrad(c, d):
    c.rows('wgrad.a', d.a, d.ntok, d.N)
    for i in range(d.n_b):
        c.rows('wgrad.b%d' % i, d.b[i], d.ntok, d.kb[i])
        ext = (d.kb[i] - 1) * d.ldo[i] + d.N if d.out_trans else (d.N - 1) * d.ldo[i] + d.kb[i]
        c.inside('wgrad.out%d' % i, d.out[i], ext * F)
    assert sum(d.kb[i] for i in range(d.n_b)) == d.Ktot
    assert d.n_split >= 1 and d.tok_per_split == 0
    c.inside('wgrad.partial', d.partial, d.n_split * d.N * d.Ktot * F)


def _attn(c, d, tag='attn'):
    D = 16 * d.H
    c.rows(tag + '.q', d.q, d.B * d.Tq, D)
    c.rows(tag + '.k', d.k, d.B * d.Tk, D)
    c.rows(tag + '.v', d.v, d.B * d.Tk, D)
    c.rows(tag + '.x', d.x, d.B * d.Tq, D)
    c.inside(tag + '.mask', d.mask, ((d.B - 1) * d.mask_sB + d.Tk) * F)
    S = d.B * d.H * d.Tq * d.Tk * F
    c.inside(tag + '.s_prev', d.s_prev, S)
    c.inside(tag + '.s_out', d.s_out, S)
    c.inside(tag + '.c', d.c, F)
    c.inside(tag + '.stats', d.stats, d.B * d.H * d.Tq * (3 if d.s_prev else 2) * F)   # + S_prev means (mep.h)


def _attn_bwd(c, d):
    f = d.f
    _attn(c, f, 'attn_bwd')
    D = 16 * f.H
    for name in ('dx', 'dq'):
        c.rows('attn_bwd.' + name, getattr(d, name), f.B * f.Tq, D)
    for name in ('dk', 'dv'):
        c.rows('attn_bwd.' + name, getattr(d, name), f.B * f.Tk, D)
    S = f.B * f.H * f.Tq * f.Tk * F
    c.inside('attn_bwd.ds_next', d.ds_next, S)
    c.inside('attn_bwd.ds_prev', d.ds_prev, S)
    c.inside('attn_bwd.dc_partial', d.dc_partial, _lib.attn_dc_slots(f.B, f.H, f.Tk) * F)


def _epi(c, d, tag='epi'):
    for name in ('q', 'x', 'xp', 'z', 'out'):
        c.rows(tag + '.' + name, getattr(d, name), d.ntok, d.D)
    c.inside(tag + '.wp', d.wp, d.D * d.D * F)
    c.inside(tag + '.wm', d.wm, 2 * d.D * d.D * F)
    c.inside(tag + '.ln_w', d.ln_w, d.D * F)
    c.inside(tag + '.ln_b', d.ln_b, d.D * F)
    c.inside(tag + '.stats', d.stats, d.ntok * 2 * F)
    c.inside(tag + '.seed', d.seed, 16)   # {seed, row0}
    if d.drop_bits:   # uint32 [ceil(ntok / 16)][2 sites][64 lanes]
        c.inside(tag + '.drop_bits', d.drop_bits, -(-d.ntok // 16) * 2 * 64 * 4)


def _epi_bwd(c, d):
    f = d.f
    _epi(c, f, 'epi_bwd')
    for name in ('dout', 'dout2', 'dz', 'dxp', 'dx', 'dq'):
        c.rows('epi_bwd.' + name, getattr(d, name), f.ntok, f.D)
    c.inside('epi_bwd.ln_partial', d.ln_partial, cdiv(f.ntok, 16) * 2 * f.D * F)
    if d.pool_T != 0:   # upstream gradient formed from the pool's dpooled / argmax slices
        assert d.dout.ptr == 0 and f.ntok % d.pool_Tq == 0
        assert d.pool_t0 + d.pool_Tq <= abs(d.pool_T) and d.pool_col + f.D <= d.pool_C and d.pool_col % 4 == 0
        nb = f.ntok // d.pool_Tq
        c.inside('epi_bwd.pool_dpooled', d.pool_dpooled, nb * 2 * d.pool_C * F)
        c.inside('epi_bwd.pool_argmax', d.pool_argmax, nb * d.pool_C * 4)


def _ln(c, d):
    for name in ('x', 'y', 'dy', 'dx'):
        c.rows('ln.' + name, getattr(d, name), d.ntok, d.D)
    c.inside('ln.w', d.w, d.D * F)
    c.inside('ln.b', d.b, d.D * F)
    c.inside('ln.stats', d.stats, d.ntok * 2 * F)
    c.inside('ln.partial', d.partial, cdiv(d.ntok, 64) * 2 * d.D * F)


def _colsum(c, d):
    c.inside('colsum.partial', d.partial, ((d.n_rows - 1) * d.ld + d.n_cols) * F)
    c.inside('colsum.out', d.out, d.n_cols * F)


def _sum(c, d):
    assert d.n_src <= _lib.SUM_MAX_SRC
    for i in range(d.n_src):
        c.rows('sum.src%d' % i, d.src[i], d.ntok, d.D)
    c.rows('sum.out', d.out, d.ntok, d.D)


def _pool(c, d):
    for name in ('x', 'dx'):
        c.inside('pool.' + name, getattr(d, name), d.B * d.T * d.C * F)
    for name in ('pooled', 'dpooled'):
        c.inside('pool.' + name, getattr(d, name), d.B * 2 * d.C * F)
    c.inside('pool.argmax', d.argmax, d.B * d.C * 4)


def _head(c, d, stride, grads):
    B, Fd, NC = d.B, d.F, d.NC
    for name in ('pooled0', 'pooled1', 'dpooled0', 'dpooled1'):
        c.inside('head.' + name, getattr(d, name), B * Fd * F)
    c.inside('head.wc0', d.wc0, NC * Fd * F)
    c.inside('head.wc1', d.wc1, NC * Fd * F)
    c.inside('head.trans', d.trans, NC ** 3 * F)
    c.inside('head.ln_w', d.ln_w, NC * F)
    c.inside('head.ln_b', d.ln_b, NC * F)
    c.inside('head.wo', d.wo, NC * 2 * NC * F)
    c.inside('head.bo', d.bo, NC * F)
    c.inside('head.labels', d.labels, B * NC * (4 if d.labels_are_float else 8))
    c.inside('head.logits', d.logits, B * NC * F)
    c.inside('head.row_loss', d.row_loss, B * F)
    c.inside('head.partial', d.partial, B * stride * F)
    if d.scale:
        c.inside('head.scale', d.scale, 2 * F)
    sizes = [NC ** 3, NC, NC, 2 * NC * NC, NC, NC * Fd, NC * Fd, 1]   # mep_head_reduce order
    for i, (gp, n) in enumerate(zip(grads, sizes)):
        c.inside('head_grad%d' % i, int(gp.value if hasattr(gp, 'value') else gp), n * F)


def _rf_epi(c, d, tag='rf_epi'):
    for name in ('q', 'x', 'xp', 'h', 'f', 'out'):
        c.rows(tag + '.' + name, getattr(d, name), d.ntok, d.D)
    c.rows(tag + '.f1', d.f1, d.ntok, d.FD)
    c.inside(tag + '.wp', d.wp, d.D * d.D * F)
    c.inside(tag + '.w1', d.w1, d.FD * d.D * F)
    c.inside(tag + '.b1', d.b1, d.FD * F)
    c.inside(tag + '.w2', d.w2, d.D * d.FD * F)
    for name in ('b2', 'ln1_w', 'ln1_b', 'ln2_w', 'ln2_b'):
        c.inside(tag + '.' + name, getattr(d, name), d.D * F)
    c.inside(tag + '.a', d.a, F)
    c.inside(tag + '.b', d.b, F)
    c.inside(tag + '.stats', d.stats, d.ntok * 4 * F)
    if d.wparts:       # wave-tiled epilogue: the six parts of Wp, W1, W2 and their transposes
        c.inside(tag + '.wparts', d.wparts, _lib.rfw_part_offsets(d.D, d.FD)[1])
    if d.wq_next:      # fused query projection of the next layer: W_q parts, QP rows
        c.inside(tag + '.wq_next', d.wq_next, _lib.wsplit_bytes(cdiv(d.D, 32) * 32, d.D))
        c.rows(tag + '.qp_next', d.qp_next, d.ntok, d.D)


def _wsplit(c, d):
    """mep_wsplit: W' [nrows][K] read from the fp32 parameter, parts written into the arena"""
    assert d.R == cdiv(d.nrows, 32) * 32 and d.nrows > 0 and d.K > 0
    ext = (d.K - 1) * d.ld + d.nrows if d.trans else (d.nrows - 1) * d.ld + d.K
    c.inside('wsplit.src', d.src, ext * F)
    c.inside('wsplit.dst', d.dst, _lib.wsplit_bytes(d.R, d.K))


def _rf_epi_bwd(c, d):
    f = d.f
    _rf_epi(c, f, 'rf_epi_bwd')
    if d.wq_in:        # fused dQP W_q input gradient of the next layer
        c.inside('rf_epi_bwd.wq_in', d.wq_in, _lib.wsplit_bytes(cdiv(f.D, 32) * 32, f.D))
        c.rows('rf_epi_bwd.dqp_in', d.dqp_in, f.ntok, f.D)
    for name in ('dout', 'dout2', 'df', 'dxp', 'dx', 'dq'):
        c.rows('rf_epi_bwd.' + name, getattr(d, name), f.ntok, f.D)
    c.rows('rf_epi_bwd.df1', d.df1, f.ntok, f.FD)
    c.inside('rf_epi_bwd.partial', d.partial, cdiv(f.ntok, _lib.rf_bwd_rows()) * _lib.rf_partial_stride(f.D, f.FD) * F)


def _rf_head(c, d):
    R, D = d.B * d.P, d.D
    for name, n in (('fc', R * D), ('h', R * D), ('dfc', R * D), ('d12', R * 12), ('ln_w', D), ('ln_b', D),
                    ('wc', 12 * D), ('bc', 12), ('trans', 36), ('out', R * 6), ('row_loss', d.B),
                    ('partial', d.B * (2 * D + 36)), ('ext_dout', R * 6)):
        c.inside('rf_head.' + name, getattr(d, name), n * F)
    c.inside('rf_head.labels', d.labels, R * 6 * 8)
    c.inside('rf_head.umask', d.umask, R * 8)
    if d.scale:
        c.inside('rf_head.scale', d.scale, F)


def check_rf_plan(p):
    c = Checker(p)
    # on the wave path (MEP_RFW, the default) the token GEMMs read mep_wsplit parts
    for arr in [p.d_unify, p.d_proj] + list(p.d_q) + list(p.d_ingrad) + [p.d_ingrad_all]:
        for d in _decode(arr):
            _gemm(c, d, parts=p.rfw)
    for arr in ([p.d_fc, p.d_fcb] if p.spec.head else []):
        for d in _decode(arr):
            _gemm(c, d)
    if p.rfw:
        for d in _decode(p.d_wsplit):
            _wsplit(c, d)
    for d in _decode(p.d_wgrad):
        _wgrad(c, d)
    for arrs, fn in ((p.d_attn, _attn), (p.d_attnb, _attn_bwd), (p.d_epi, _rf_epi), (p.d_epib, _rf_epi_bwd)):
        for arr in arrs:
            for d in _decode(arr):
                fn(c, d)
    for d in _decode(p.d_colsum):
        _colsum(c, d)
    for d in _decode(p.d_sum):
        _sum(c, d)
    for d in _decode(getattr(p, 'd_isum', None)):
        # mep_wgemm_sum: every source GEMM's rows and parts, then the sum's output rows
        assert 1 <= d.n_src <= _lib.WGEMM_SUM_MAX
        for i in range(d.n_src):
            _gemm(c, d.src[i], parts=True)
            assert d.src[i].ntok == d.src[0].ntok and d.src[i].N == d.src[0].N
        c.rows('wgemm_sum.out', d.out, d.src[0].ntok, d.src[0].N)
    if p.spec.head:
        for d in _decode(p.d_pool):
            _pool(c, d)
        _rf_head(c, p.head)
    return c.n


def check_plan(p):
    c = Checker(p)
    for d in _decode(p.d_unify):
        _gemm(c, d)
    for d in _decode(p.d_wgrad):
        _wgrad(c, d)
    for arrs, fn in ((p.d_attn, _attn), (p.d_attnb, _attn_bwd), (p.d_epi, _epi), (p.d_epib, _epi_bwd)):
        for arr in arrs:
            for d in _decode(arr):
                fn(c, d)
    for name in ('d_uln', 'd_ulnb'):
        for d in _decode(getattr(p, name, None)):
            _ln(c, d)
    for name in ('d_colsum', 'd_losssum'):
        for d in _decode(getattr(p, name)):
            _colsum(c, d)
    for d in _decode(p.d_sum):
        _sum(c, d)
    for d in _decode(p.d_pool):
        _pool(c, d)
    _head(c, p.head, p.head_stride, p.head_grads)
    return c.n


CASES = [
    ('cmu', dict(dim=32, n_heads=2, n_layers=1), 5, (7, 9, 12)),
    ('cmu', dict(dim=32, n_heads=2, n_layers=2), 4, (6, 10, 8)),
    ('cmu', dict(dim=96, n_heads=6, n_layers=1), 3, (50, 50, 50)),
    ('cmu', dict(dim=64, n_heads=4, n_layers=3), 2, (1, 65, 130)),
    ('ren', dict(dim=32, n_heads=2, n_layers=1), 6, (5, 6, 8)),
    ('ren', dict(dim=128, n_heads=8, n_layers=1), 2, (40, 76, 275)),
    ('ren', dict(dim=64, n_heads=4, n_layers=2), 4, (3, 70, 9)),
]


@pytest.mark.parametrize('bf16', [False, True], ids=['fp32', 'bf16'])
@pytest.mark.parametrize('family,kw,B,T', CASES)
def test_plan_descriptors_in_bounds(family, kw, B, T, bf16):
    from mep_amd import cmu_mosei, ren_mme
    Tl, Tv, Ta = T
    if family == 'cmu':
        m = cmu_mosei.Concat_Trans(kw['dim'], Tl, Tv, Ta, kw['n_heads'], kw['n_layers'], 1)
    else:
        m = ren_mme.Base_model(dim=kw['dim'], l_len=Tl, v_len=Tv, a_len=Ta, n_heads=kw['n_heads'],
                               n_layers=kw['n_layers'])
    runner = m.mep_runner('cpu')
    plan = runner.plan(B, T, bf16=bf16)
    n = check_plan(plan)
    assert n > 50
    assert len(plan.blocks) == 18 * kw['n_layers']
    if bf16:
        _check_bf16_views(plan)


def _check_bf16_views(plan):
    """The bf16 path's storage contract (include/mep.h MEP_PREC_BF16): every activation view the
    bf16 kernels read or write as bf16 points into a bf16 buffer, the pooled tensor, scores and
    statistics into fp32 ones -- a view into a buffer of the other width would be read as garbage."""
    c = Checker(plan)
    half = lambda r: r.ptr == 0 or c.elsize(r.ptr) == 2     # noqa: E731
    full = lambda r: r.ptr == 0 or c.elsize(r.ptr) == 4     # noqa: E731
    for d in _decode(plan.d_unify):
        assert d.bf16 == 3 and half(d.x) and half(d.y)
    for arr in plan.d_attn:
        for d in _decode(arr):
            assert all(half(getattr(d, k)) for k in ('q', 'k', 'v', 'x'))
    for arr in plan.d_attnb:
        for d in _decode(arr):
            assert all(half(getattr(d, k)) for k in ('dx', 'dq', 'dk', 'dv'))
    for arr in plan.d_epi:
        for d in _decode(arr):
            assert all(half(getattr(d, k)) for k in ('q', 'x', 'xp', 'z', 'out_h')) and full(d.out)
    for arr in plan.d_epib:
        for d in _decode(arr):
            assert all(half(getattr(d, k)) for k in ('dout2', 'dz', 'dxp', 'dx', 'dq'))
    for d in _decode(plan.d_wgrad):
        assert d.bf16 == 3 and half(d.a) and all(half(d.b[i]) for i in range(d.n_b))
    for d in _decode(plan.d_sum):
        assert d.accumulate == 2 and half(d.out) and all(half(d.src[i]) for i in range(d.n_src))
    for name in ('d_uln', 'd_ulnb'):
        for d in _decode(getattr(plan, name, None)):
            assert d.bf16 == 2 and all(half(getattr(d, k)) for k in ('x', 'y', 'dy', 'dx'))


RF_CASES = [
    (dict(dim=32, n_heads=2, n_layers=2, T=6, ffn=2), 3, 3, True),
    (dict(dim=96, n_heads=6, n_layers=2, T=50, ffn=2), 2, 6, True),
    (dict(dim=64, n_heads=4, n_layers=1, T=70, ffn=1), 2, 2, True),
    (dict(dim=96, n_heads=6, n_layers=2, T=50, ffn=2), 4, 1, False),
]


@pytest.mark.parametrize('kw,B,P,head', RF_CASES)
def test_realformer_plan_descriptors_in_bounds(kw, B, P, head):
    from mep_amd import realformer as rf
    old = rf.FFN
    rf.FFN = kw['ffn']
    try:
        T = kw['T']
        if head:
            m = rf.State_Transfer(300, 35, 74, kw['dim'], T, T, T, kw['n_heads'], kw['n_layers'], kw['ffn'])
            plan = m.mep_runner('cpu').plan(B, P)
        else:
            m = rf.Multi_class(300, 35, 74, kw['dim'], T, T, T, kw['n_heads'], kw['n_layers'], kw['ffn'])
            plan = m.mep_chain_runner(kw['n_layers'], 'cpu').plan(B, 1)
    finally:
        rf.FFN = old
    assert check_rf_plan(plan) > 20
    # the cfg2 chain's input gradients run fused with their per-modality sum (<= 4 sources per
    # sum); State_Transfer's sums have 9 sources and keep the two launches
    assert (plan.d_isum is not None) == (not head)


def test_row_views_within_24_bit_addressing():
    """include/mep.h mep_rows: strides below 2^24 elements (the kernels' 24-bit row addressing);
    a host view past that is refused when it is built, not mis-addressed on the GPU"""
    from mep_amd.trimodal import rows
    t = torch.zeros(8, 4)
    assert rows(t, 2, 8, 4).sB == 8
    with pytest.raises(ValueError):
        rows(t, 2, 1 << 24, 4)
    with pytest.raises(ValueError):
        rows(t, 2, 8, 1 << 24)


def _writes(arr_w, arr_c, head=None, NC=None, Fd=None):
    """(first float, count) runs of the flat gradient buffer a bucket's launches write: the weight
    gradients' output rows, the column sums and the fused head's parameter sums"""
    out = []
    for d in (arr_w.items if arr_w is not None else []):
        for b in range(d.n_b):
            rows_, cols_ = (d.kb[b], d.N) if d.out_trans else (d.N, d.kb[b])
            out += [(d.out[b] + 4 * r * d.ldo[b], cols_) for r in range(rows_)]
    for c in (arr_c.items if arr_c is not None else []):
        out.append((c.out, c.n_cols))
    if head is not None:
        sizes = [NC ** 3, NC, NC, 2 * NC * NC, NC, NC * Fd, NC * Fd]   # mep_head_reduce order
        out += [(int(p), n) for p, n in zip(head, sizes)]
    return out


@pytest.mark.parametrize('family,kw,B,T', CASES)
def test_gradient_buckets_partition_the_flat_gradient(family, kw, B, T):
    """The data-parallel exchange all-reduces flat.grad[:split] (bucket A) on a side stream while
    bucket B's launches still run (engine.py).  Every gradient element must be written by exactly
    one launch of exactly the bucket whose all-reduce covers it, and nothing outside [0, n_grad)
    may be written -- else a gradient would be summed before it is final, or never."""
    from mep_amd import cmu_mosei, ren_mme
    Tl, Tv, Ta = T
    if family == 'cmu':
        m = cmu_mosei.Concat_Trans(kw['dim'], Tl, Tv, Ta, kw['n_heads'], kw['n_layers'], 1)
    else:
        m = ren_mme.Base_model(dim=kw['dim'], l_len=Tl, v_len=Tv, a_len=Ta, n_heads=kw['n_heads'],
                               n_layers=kw['n_layers'])
    plan = m.mep_runner('cpu').plan(B, T)
    plan._build_buckets()          # asserts every write range against its bucket (_check_bucket_ranges)
    (_, wa, _, _), (_, wb, _, _), ca, cb = plan._buckets
    fl = plan.flat
    g0 = fl.grad.data_ptr()
    count = torch.zeros(fl.total, dtype=torch.int32)
    owner = torch.full((fl.total,), -1, dtype=torch.int32)
    NC, Fd = plan.spec.NC, plan.F
    for k, (w, c, head) in enumerate(((wa, ca, plan.head_grads[:-1]), (wb, cb, None))):
        for ptr, n in _writes(w, c, head, NC, Fd):
            assert (ptr - g0) % 4 == 0
            o = (ptr - g0) // 4
            assert 0 <= o and o + n <= fl.n_grad, (k, o, n, fl.n_grad)
            count[o:o + n] += 1
            owner[o:o + n] = k
    for name in fl.names:
        o, n = fl.offsets[name], fl.params[name].numel()
        if not fl.has_grad[name]:
            assert int(count[o:o + n].sum()) == 0, name
            continue
        assert bool((count[o:o + n] == 1).all()), (name, count[o:o + n].min(), count[o:o + n].max())
        want = 0 if o < fl.split else 1
        assert bool((owner[o:o + n] == want).all()), (name, 'written by the other bucket')
    # the same launches, unsplit, write the same elements (backward() without the exchange)
    full = torch.zeros(fl.total, dtype=torch.int32)
    for ptr, n in _writes(plan.d_wgrad, plan.d_colsum, plan.head_grads[:-1], NC, Fd):
        o = (ptr - g0) // 4
        full[o:o + n] += 1
    assert torch.equal(full, count)


def test_wgemm_ws_only_within_its_k_limit():
    """mep_wgemm_ws keeps a column block's parts of every k pair in LDS and refuses K > 320
    (rfw.hip mep_wgemm_ws); a large launch with a wider feature dim goes to mep_wgemm"""
    from types import SimpleNamespace as NS
    big = [NS(ntok=19200, N=96, K=300), NS(ntok=19200, N=96, K=74), NS(ntok=19200, N=96, K=35)]
    assert _lib.wgemm_tiles(big) >= _lib.WGEMM_WS_MIN
    assert _lib.wgemm_ws_fits(big) == _lib.WGEMM_WS
    wide = [NS(ntok=19200, N=96, K=400)] + big[1:]
    assert not _lib.wgemm_ws_fits(wide)
    small = [NS(ntok=3200, N=96, K=300)]
    assert not _lib.wgemm_ws_fits(small)


def _check_reduce_map(bmap, wgrad, colsum, head):
    """a mep_reduce_grads_mapped job list: every real job once, nothing else"""
    import numpy as np
    m, n = bmap
    jobs = m.cpu().numpy().view(np.uint32)[:n]
    want = set()
    if head is not None:
        want |= {(0, 0, j) for j in range(_lib.lib().mep_reduce_grads_grid(0, 0, 0, 0, ctypes.byref(head)))}
    for i, d in enumerate(wgrad.items):
        want |= {(1, i, b) for b in range(cdiv(d.N * d.Ktot, 1024))}
    for i, c in enumerate(colsum.items if colsum is not None else []):
        want |= {(2, i, b) for b in range(cdiv(c.n_cols, 32))}
    got = [(int(j) >> 30, (int(j) >> 12) & 0x3ffff, int(j) & 0xfff) for j in jobs]
    assert len(got) == len(set(got)) == len(want) and set(got) == want


def test_reduce_maps_list_every_real_job():
    """the compact block maps of the gradient reduction (trimodal.reduce_map): cfg3 (one launch and
    the two data-parallel buckets) and State_Transfer, whose rectangular grid was 29,430 blocks"""
    from mep_amd import cmu_mosei
    from mep_amd import realformer as rf, rf_plan
    p = cmu_mosei.Concat_Trans(96, 50, 50, 50, 6, 1, 1).mep_runner('cpu').plan(64, (50, 50, 50))
    _check_reduce_map(p.redmap, p.d_wgrad, p.d_colsum, p.head)
    assert p.redmap[1] < p.reduce_grid() + 1 and p.redmap[1] < 1377
    p._build_buckets()
    (_, da, _, _), (_, db, _, _), ca, cb = p._buckets
    _check_reduce_map(p._bucket_maps[0], da, ca, p.head)
    _check_reduce_map(p._bucket_maps[1], db, cb, None)
    st = rf.State_Transfer(300, 35, 74, 96, 50, 50, 50, 6, 2, 2)
    r = st.mep_runner('cpu')
    q = rf_plan.RealformerPlan(r.spec, r.flat, 64, 6, 'cpu')
    _check_reduce_map(q.redmap, q.d_wgrad, q.d_colsum, None)
    assert q.reduce_grid() == q.redmap[1] < 3000
