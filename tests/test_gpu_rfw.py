"""The wave-tiled realformer kernels (csrc/rfw.hip) against float64 torch statements:

* mep_wsplit: the three bf16 parts of a weight (and of its transpose, with rows padded to 32 and
  K padded to 32) sum back to the fp32 weight within 2^-24 relative, in the unit order the
  kernels read (unit (n, p, g) = W(n, 32p + 4g .. +3) then W(n, 32p + 16 + 4g .. +3));
* mep_wgemm: the mep_gemm contract on pre-split weights -- the realformer Conv1d unify with a
  position table and K = 300 (others/realformer.py:136-152,224-227), w_qkv with N = 2D = 192
  (realformer.py:157), the dY W input-gradient form on the parts of W^T accumulating onto y,
  unaligned K (scalar X loads), bias + relu, ragged token counts;
* mep_rfw_epi_fwd with the fused next-layer query projection: out against a float64 statement of
  realformer.py:203-209, and qp_next against out Wq^T in float64.
Six bf16 products per k pair are fp32-level: rtol 1e-5, atol 1e-6 of max|y|."""
import pytest
import torch

from tests.gpu_util import assert_close

pytestmark = pytest.mark.gpu


def _rows(t, T, sB, sT, off=0):
    from mep_amd._lib import Rows
    return Rows(ptr=t.data_ptr() + 4 * off, sB=sB, sT=sT, T=T)


def _parts(ws, dev):
    """mep_wsplit of [(W, N, K, ld, trans)] into one arena; returns (buffer, offsets)"""
    from mep_amd import _lib
    arena = _lib.PartsArena()
    offs = [arena.add(w.data_ptr(), N, K, ld, trans) for (w, N, K, ld, trans) in ws]
    buf, descs, units = arena.build(dev)
    _lib.launch('mep_wsplit', descs, units)
    torch.cuda.synchronize()
    return buf, offs


def _unsplit(buf, off, R, K):
    """float64 sum of the three parts of an R x K weight at byte offset off, as [R][Kp]"""
    npk = -(-K // 32)
    n_units = R * npk * 4
    raw = buf[off:off + 3 * n_units * 16].view(torch.int16).view(3, R, npk, 4, 8)
    f = ((raw.to(torch.int64) & 0xFFFF) << 16).to(torch.int32).view(torch.float32).double()   # bf16 -> f32 bits
    parts = f.sum(0)                                                 # [R][npk][4 g][8]
    lo, hi = parts[..., :4], parts[..., 4:]                          # k = 32p + 4g + e, +16
    out = torch.zeros(R, npk, 32, dtype=torch.float64, device=buf.device)
    for g in range(4):
        out[:, :, 4 * g:4 * g + 4] = lo[:, :, g]
        out[:, :, 16 + 4 * g:16 + 4 * g + 4] = hi[:, :, g]
    return out.reshape(R, npk * 32)


@pytest.mark.parametrize('N,K', [(96, 300), (192, 96), (80, 35), (96, 192)])
def test_wsplit_round_trip(N, K, cuda):
    torch.manual_seed(N + K)
    w = torch.randn(N, K, device=cuda)
    buf, (o_w, o_t) = _parts([(w, N, K, K, 0), (w, K, N, K, 1)], cuda)   # W [N][K] and W^T [K][N]
    R, RT = -(-N // 32) * 32, -(-K // 32) * 32
    got = _unsplit(buf, o_w, R, K)
    want = torch.zeros_like(got)
    want[:N, :K] = w.double()
    assert_close(got, want.cpu().numpy(), 2 ** -24, 0, 'W parts')
    got_t = _unsplit(buf, o_t, RT, N)
    want_t = torch.zeros_like(got_t)
    want_t[:K, :N] = w.double().t()
    assert_close(got_t, want_t.cpu().numpy(), 2 ** -24, 0, 'W^T parts')


def _wgemm(descs, dev):
    from mep_amd import _lib
    arr = _lib.DescArray(_lib.GemmDesc, descs, dev)
    tiles = max(-(-d.ntok // 16) for d in descs)
    _lib.call('mep_wgemm', arr.ptr, arr.n, tiles, max(d.N for d in descs))
    torch.cuda.synchronize()


def _gd(x, y, w, ntok, N, K, bias=None, table=None, accumulate=0, relu=0, alpha=1.0, ldt=0):
    from mep_amd._lib import GemmDesc
    return GemmDesc(x=x, y=y, w=w, bias=bias.data_ptr() if bias is not None else 0,
                    table=table.data_ptr() if table is not None else 0, ntok=ntok, N=N, K=K, ldw=0, w_nt=1,
                    accumulate=accumulate, relu=relu, alpha=alpha, bf16=0, ldt=ldt)


@pytest.mark.parametrize('B,T', [(64, 50), (3, 7)])
def test_wgemm_vs_float64(B, T, cuda):
    torch.manual_seed(B * T)
    D = 96
    # Conv1d unify (K = 300) + position table, w_qkv [K | V] (N = 2D), dY W (parts of W^T,
    # accumulating), an unaligned K = 35 with bias + relu
    x = torch.randn(B, T, 300, device=cuda)
    wu = torch.randn(D, 300, device=cuda) / 300 ** 0.5
    pos = torch.randn(T, D, device=cuda)
    u = torch.randn(B * T, D, device=cuda)
    wkv = torch.randn(2 * D, D, device=cuda) / D ** 0.5
    dy = torch.randn(B * T, 2 * D, device=cuda)
    y0 = torch.randn(B * T, D, device=cuda)
    x35 = torch.randn(B, T, 35, device=cuda)
    w35 = torch.randn(D, 35, device=cuda) / 35 ** 0.5
    bias = torch.randn(D, device=cuda)
    buf, (o_u, o_kv, o_t, o_35) = _parts([(wu, D, 300, 300, 0), (wkv, 2 * D, D, D, 0), (wkv, D, 2 * D, D, 1),
                                          (w35, D, 35, 35, 0)], cuda)
    base = buf.data_ptr()
    yu = torch.zeros(B * T, D, device=cuda)
    ykv = torch.zeros(B * T, 2 * D, device=cuda)
    yin = y0.clone()
    y35 = torch.zeros(B * T, D, device=cuda)
    n = B * T
    _wgemm([_gd(_rows(x, T, T * 300, 300), _rows(yu, T, T * D, D), base + o_u, n, D, 300, table=pos),
            _gd(_rows(u, T, T * D, D), _rows(ykv, T, T * 2 * D, 2 * D), base + o_kv, n, 2 * D, D),
            _gd(_rows(dy, T, T * 2 * D, 2 * D), _rows(yin, T, T * D, D), base + o_t, n, D, 2 * D, accumulate=1),
            _gd(_rows(x35, T, T * 35, 35), _rows(y35, T, T * D, D), base + o_35, n, D, 35, bias=bias, relu=1)],
           cuda)
    ref_u = (x.double().reshape(n, 300) @ wu.double().t()).reshape(B, T, D) + pos.double()
    assert_close(yu.reshape(B, T, D), ref_u.cpu().numpy(), 1e-5, 1e-6, 'unify + table')
    assert_close(ykv, (u.double() @ wkv.double().t()).cpu().numpy(), 1e-5, 1e-6, 'w_qkv')
    assert_close(yin, (y0.double() + dy.double() @ wkv.double()).cpu().numpy(), 1e-5, 1e-6, 'dY W (+= y)')
    ref35 = torch.relu(x35.double().reshape(n, 35) @ w35.double().t() + bias.double())
    assert_close(y35, ref35.cpu().numpy(), 1e-5, 1e-6, 'K = 35, bias + relu')


def _wgemm_ws(descs, dev):
    from mep_amd import _lib
    _lib.wgemm_ws(_lib.DescArray(_lib.GemmDesc, descs, dev))
    torch.cuda.synchronize()


# descriptor mixes of one launch -> the LDS-resident instance (column tiles NT, k pairs NPK) the
# host picks: rfstate-sized w_qkv (12, 3), the input gradients (6, 6), unify K = 300 (3, 10),
# small launches narrowing the column block (3, 3), (3, 6), ragged N / K and a single tile
WS_CASES = {
    'qkv_big': (64 * 6 * 50, [(96, 192, 0), (96, 96, 0)]),
    'ingrad': (64 * 6 * 50, [(96, 96, 1), (192, 96, 1)]),
    'unify': (32 * 6 * 50, [(300, 96, 0), (35, 96, 0), (74, 96, 0)]),
    'small': (50 * 3, [(96, 192, 0), (96, 96, 0)]),
    'small_k192': (50 * 3, [(192, 96, 1)]),
    'ragged': (37, [(70, 42, 1), (33, 18, 0)]),
}


@pytest.mark.parametrize('case', sorted(WS_CASES))
def test_wgemm_ws_matches_wgemm(case, cuda):
    """mep_wgemm_ws == mep_wgemm bit for bit (same products, same order) and both within fp32
    level of float64: every (K, N, accumulate) descriptor of the case in one launch; the
    bias / table / relu epilogue on the first descriptor."""
    n, shapes = WS_CASES[case]
    torch.manual_seed(len(case) * 1000 + n)
    T = 50 if n % 50 == 0 else n
    ws, xs, ys, y0s = [], [], [], []
    for (K, N, acc) in shapes:
        ws.append((torch.randn(N, K, device=cuda) / K ** 0.5, N, K, K, 0))
        xs.append(torch.randn(n, K, device=cuda))
        y0s.append(torch.randn(n, N, device=cuda) if acc else torch.zeros(n, N, device=cuda))
    bias = torch.randn(shapes[0][1], device=cuda)
    table = torch.randn(T, shapes[0][1], device=cuda)
    buf, offs = _parts(ws, cuda)
    outs = []
    for run in (_wgemm, _wgemm_ws):
        ys = [y.clone() for y in y0s]
        descs = []
        for i, ((K, N, acc), x, y, o) in enumerate(zip(shapes, xs, ys, offs)):
            extra = dict(bias=bias, table=table, relu=1) if i == 0 else {}
            descs.append(_gd(_rows(x, T, T * K, K), _rows(y, T, T * N, N), buf.data_ptr() + o, n, N, K,
                             accumulate=acc, **extra))
        run(descs, cuda)
        outs.append(ys)
    for i, ((K, N, acc), x, y0, (w, *_)) in enumerate(zip(shapes, xs, y0s, ws)):
        a, b = outs[0][i], outs[1][i]
        assert torch.equal(a, b), '%s desc %d: max |diff| %.3g' % (case, i, (a - b).abs().max().item())
        ref = x.double() @ w.double().t()
        if i == 0:
            ref = torch.relu(ref + bias.double() + table.double().repeat(n // T, 1))
        if acc:
            ref = ref + y0.double()
        assert_close(b, ref.cpu().numpy(), 1e-5, 1e-6, '%s desc %d' % (case, i))


def test_rfw_fused_query_projection(cuda):
    """qp_next from the fused epilogue tail equals out Wq^T (float64) of the same launch's out."""
    from mep_amd import _lib
    from mep_amd._lib import DescArray, RfEpiDesc
    from mep_amd.trimodal import crows
    torch.manual_seed(5)
    B, T, D, FD = 8, 50, 96, 192
    n = B * T
    f = dict(device=cuda, dtype=torch.float32)
    q, x = torch.randn(n, D, **f), torch.randn(n, D, **f)
    xp, h, f_, out, qp = (torch.zeros(n, D, **f) for _ in range(5))
    f1 = torch.zeros(n, FD, **f)
    stats = torch.zeros(n, 4, **f)
    wp = torch.randn(D, D, **f) / D ** 0.5
    w1 = torch.randn(FD, D, **f) / D ** 0.5
    w2 = torch.randn(D, FD, **f) / FD ** 0.5
    wq = torch.randn(D, D, **f) / D ** 0.5
    vec = lambda m: torch.randn(m, **f)  # noqa: E731
    b1, b2, l1w, l1b, l2w, l2b = vec(FD), vec(D), vec(D), vec(D), vec(D), vec(D)
    a, bb = torch.tensor([0.7], **f), torch.tensor([-0.3], **f)
    arena = _lib.PartsArena()
    o_epi = arena.add_epi(D, FD, wp.data_ptr(), w1.data_ptr(), w2.data_ptr())
    o_q = arena.add(wq.data_ptr(), D, D, D, 0)
    buf, wsd, units = arena.build(cuda)
    _lib.launch('mep_wsplit', wsd, units)
    ed = RfEpiDesc(q=crows(q, T, D), x=crows(x, T, D), xp=crows(xp, T, D), h=crows(h, T, D), f1=crows(f1, T, FD),
                   f=crows(f_, T, D), out=crows(out, T, D), wp=wp.data_ptr(), w1=w1.data_ptr(), b1=b1.data_ptr(),
                   w2=w2.data_ptr(), b2=b2.data_ptr(), ln1_w=l1w.data_ptr(), ln1_b=l1b.data_ptr(),
                   ln2_w=l2w.data_ptr(), ln2_b=l2b.data_ptr(), a=a.data_ptr(), b=bb.data_ptr(),
                   stats=stats.data_ptr(), ntok=n, D=D, FD=FD, wparts=buf.data_ptr() + o_epi,
                   wq_next=buf.data_ptr() + o_q, qp_next=crows(qp, T, D))
    _lib.launch('mep_rfw_epi_fwd', DescArray(RfEpiDesc, [ed], cuda), -(-n // 16), extra=(D, FD))
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert_close(qp, (out.double() @ wq.double().t()).cpu().numpy(), 1e-5, 1e-6, 'qp_next')
    # the epilogue itself against a float64 statement of realformer.py:203-209
    dd = lambda t: t.double()  # noqa: E731
    xp_r = dd(x) @ dd(wp).t()
    z1 = dd(q) + dd(a) * xp_r
    h_r = torch.nn.functional.layer_norm(z1, (D,), dd(l1w), dd(l1b), 1e-5)
    f1_r = torch.relu(h_r @ dd(w1).t() + dd(b1))
    f_r = f1_r @ dd(w2).t() + dd(b2)
    out_r = torch.nn.functional.layer_norm(h_r + dd(bb) * f_r, (D,), dd(l2w), dd(l2b), 1e-5)
    assert_close(out, out_r.cpu().numpy(), 1e-4, 1e-6, 'out')
    assert_close(f1, f1_r.cpu().numpy(), 1e-4, 1e-6, 'f1')


@pytest.mark.parametrize('family', ['chain', 'state'])
def test_rfw_front_matches_gemm_launches(family, cuda):
    """mep_rfw_front (unify + every projection of U in one launch per modality) writes U, [K | V]
    and the layer-0 Q bit-identical to the mep_wgemm / mep_wgemm_ws launches it replaces: the
    cfg2 text chain (d = 300) and a State_Transfer plan (d = 300 / 35 / 74, three launches)."""
    from mep_amd import realformer as rf
    from mep_amd import rf_plan
    torch.manual_seed(11)
    B, P, T = 8, 3, 50
    if family == 'chain':
        mc = rf.Multi_class(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=T, v_len=T, a_len=T, n_heads=6,
                            n_layers=2, ffn=2).to(cuda)
        runner, PP = mc.mep_chain_runner(2, cuda), 1
        feats = (torch.randn(B, T, 300, device=cuda), torch.zeros(0, device=cuda), torch.zeros(0, device=cuda))
        masks = (torch.ones(B, T, device=cuda), torch.zeros(0, device=cuda), torch.zeros(0, device=cuda))
    else:
        st = rf.State_Transfer(300, 35, 74, 96, T, T, T, 6, 2, 2).to(cuda)
        runner, PP = st.mep_runner(cuda), P
        feats = tuple(torch.randn(B, P, T, d, device=cuda) for d in (300, 35, 74))
        masks = tuple((torch.rand(B, P, T, device=cuda) > 0.2).float() for _ in range(3))
    outs = []
    for on in (True, False):
        old = rf_plan.RF_FRONT, rf_plan.RF_FRONT_MAX_TILES
        rf_plan.RF_FRONT, rf_plan.RF_FRONT_MAX_TILES = on, 1 << 30
        try:
            plan = rf_plan.RealformerPlan(runner.spec, runner.flat, B, PP, cuda)
        finally:
            rf_plan.RF_FRONT, rf_plan.RF_FRONT_MAX_TILES = old
        assert bool(plan.front) == on
        plan.set_inputs(*feats, *masks)
        plan.forward(grad=False)
        torch.cuda.synchronize()
        outs.append([plan.U[m].clone() for m in plan.spec.mods] +
                    [b['KV'].clone() for b in plan.blocks] + [b['QP'].clone() for b in plan.blocks if b['i'] == 0])
    for i, (a, b) in enumerate(zip(*outs)):
        assert torch.equal(a, b), 'tensor %d: max |diff| %.3g' % (i, (a - b).abs().max().item())


def _sum_rows(srcs, out, ntok, D, dev):
    from mep_amd import _lib
    src = (_lib.Rows * _lib.SUM_MAX_SRC)(*srcs)
    arr = _lib.DescArray(_lib.SumDesc, [_lib.SumDesc(src=src, out=out, n_src=len(srcs), ntok=ntok, D=D,
                                                    accumulate=0)], dev)
    _lib.call('mep_sum_rows', arr.ptr, arr.n, min(1024, -(-ntok * D // 1024)))
    torch.cuda.synchronize()


# (tokens, T, [(K, accumulate) per source]) of one fused sum: cfg2's chain modality (layer-0
# dq_in onto the epilogue residual + two dkv_in), four sources, one source, ragged tokens
SUM_CASES = {
    'chain': (64 * 50, 50, [(96, 1), (192, 0), (192, 0)]),
    'four': (8 * 50, 50, [(192, 0), (96, 1), (192, 1), (35, 0)]),
    'one': (3 * 7, 7, [(96, 1)]),
    'ragged': (37, 37, [(70, 0), (192, 1)]),
}


@pytest.mark.parametrize('case', sorted(SUM_CASES))
def test_wgemm_sum_matches_wgemm_and_sum_rows(case, cuda):
    """mep_wgemm_sum == mep_wgemm per source + mep_sum_rows bit for bit, the sources' y rows
    untouched, and within fp32 level of the float64 sum of products."""
    from mep_amd import _lib
    n, T, shapes = SUM_CASES[case]
    D = 96
    torch.manual_seed(n + len(shapes))
    ws = [(torch.randn(D, K, device=cuda) / K ** 0.5, D, K, K, 0) for K, _ in shapes]
    xs = [torch.randn(n, K, device=cuda) for K, _ in shapes]
    y0s = [torch.randn(n, D, device=cuda) if acc else torch.zeros(n, D, device=cuda) for _, acc in shapes]
    buf, offs = _parts(ws, cuda)

    def descs(ys):
        return [_gd(_rows(x, T, T * K, K), _rows(y, T, T * D, D), buf.data_ptr() + o, n, D, K, accumulate=acc)
                for (K, acc), x, y, o in zip(shapes, xs, ys, offs)]

    ys = [y.clone() for y in y0s]
    _wgemm(descs(ys), cuda)
    want = torch.full((n, D), float('nan'), device=cuda)
    _sum_rows([_rows(y, T, T * D, D) for y in ys], _rows(want, T, T * D, D), n, D, cuda)
    ys2 = [y.clone() for y in y0s]
    got = torch.full((n, D), float('nan'), device=cuda)
    src = (_lib.GemmDesc * _lib.WGEMM_SUM_MAX)(*descs(ys2))
    arr = _lib.DescArray(_lib.GemmSumDesc, [_lib.GemmSumDesc(src=src, n_src=len(shapes),
                                                             out=_rows(got, T, T * D, D))], cuda)
    _lib.call('mep_wgemm_sum', arr.ptr, arr.n, -(-n // 16), D)
    torch.cuda.synchronize()
    assert torch.equal(got, want), '%s: max |diff| %.3g' % (case, (got - want).abs().max().item())
    for y, y0 in zip(ys2, y0s):
        assert torch.equal(y, y0)
    ref = sum(x.double() @ w.double().t() + y0.double() for x, y0, (w, *_) in zip(xs, y0s, ws))
    assert_close(got, ref.cpu().numpy(), 1e-5, 1e-6, case)


def test_rfw_wgemm_sum_plan_gradients(cuda):
    """cfg2's text chain: the backward with the fused input-gradient sums (mep_wgemm_sum) writes
    every gradient bit-identical to the ingrad GEMM + mep_sum_rows launches."""
    from mep_amd import realformer as rf
    from mep_amd import rf_plan
    torch.manual_seed(12)
    B, T = 8, 50
    mc = rf.Multi_class(l_dim=300, v_dim=35, a_dim=74, dim=96, l_len=T, v_len=T, a_len=T, n_heads=6,
                        n_layers=2, ffn=2).to(cuda)
    runner = mc.mep_chain_runner(2, cuda)
    feats = (torch.randn(B, T, 300, device=cuda), torch.zeros(0, device=cuda), torch.zeros(0, device=cuda))
    masks = (torch.ones(B, T, device=cuda), torch.zeros(0, device=cuda), torch.zeros(0, device=cuda))
    dout = None
    grads = []
    for on in (True, False):
        old = rf_plan.RF_WGEMM_SUM
        rf_plan.RF_WGEMM_SUM = on
        try:
            plan = rf_plan.RealformerPlan(runner.spec, runner.flat, B, 1, cuda)
        finally:
            rf_plan.RF_WGEMM_SUM = old
        assert (plan.d_isum is not None) == on
        plan.set_inputs(*feats, *masks)
        plan.forward(grad=True)
        if dout is None:
            dout = torch.randn_like(plan.dout_chain)
        runner.flat.grad.zero_()
        plan.backward(ext_dout=dout)
        torch.cuda.synchronize()
        grads.append(runner.flat.grad.clone())
    assert torch.equal(grads[0], grads[1]), 'max |diff| %.3g' % (grads[0] - grads[1]).abs().max().item()


@pytest.mark.parametrize('B,P', [(16, 6), (13, 5)])
def test_rfs_matches_per_tile_epilogues(B, P, cuda, monkeypatch):
    """The weight-stationary State_Transfer epilogue launches (k_rfs_fwd / k_rfs_bwd, on by default
    for >= MEP_RFW_BIG_TILES tiles) write the logits, every block output and every gradient
    (and the epilogue rows h / f1 / f / out / the fused next-layer q of every block) bit-identical
    to the per-tile kernels they replace (MEP_RFS=0): same products in the same
    order, same epilogue arithmetic.  13 x 5 x 50 tokens per block: a ragged last tile and a
    last job with idle waves."""
    from mep_amd import realformer as rf
    from mep_amd import rf_plan
    torch.manual_seed(B * P)
    T = 50
    st = rf.State_Transfer(300, 35, 74, 96, T, T, T, 6, 2, 2).to(cuda)
    runner = st.mep_runner(cuda)
    feats = tuple(torch.randn(B, P, T, d, device=cuda) for d in (300, 35, 74))
    masks = tuple((torch.rand(B, P, T, device=cuda) > 0.2).float() for _ in range(3))
    dout = torch.randn(B, P, 6, device=cuda)
    res = []
    for on in ('1', '0'):
        monkeypatch.setenv('MEP_RFS', on)
        plan = rf_plan.RealformerPlan(runner.spec, runner.flat, B, P, cuda)
        for i in range(plan.spec.nl):   # every epilogue launch takes the large-launch path
            assert plan.t_epif[i] * plan.d_epi[i].n >= 1024
        plan.set_inputs(*feats, *masks)
        plan.forward(grad=True)
        runner.flat.grad.zero_()
        plan.backward(ext_dout=dout)
        torch.cuda.synchronize()
        res.append([plan.out.clone(), runner.flat.grad.clone()] +
                   [b[k].clone() for b in plan.blocks for k in ('H', 'F1', 'F', 'OUT', 'QP') if k in b])
    assert torch.isfinite(res[0][0]).all() and torch.isfinite(res[0][1]).all()
    for i, (a, b) in enumerate(zip(*res)):
        assert torch.equal(a, b), 'tensor %d: max |diff| %.3g' % (i, (a - b).abs().max().item())
