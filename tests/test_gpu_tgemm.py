"""mep_tgemm (csrc/tgemm.hip k_tgemm, the tiled split-bf16 token GEMM) against a float64 torch
statement of the mep_gemm contract: the Unify_Dimension Linears (cmu-mosei/run.py:210-214,
Ren-MME/run.py:161-166) on slot views of [B, 2, T, d] inputs with unaligned K (35, 74, 205: scalar
X loads) and ragged token counts, the realformer Conv1d unify + position table
(others/realformer.py:136-152), w_qkv with N = 2D = 192 (two N tiles), the input-gradient form
with W stored [K][N] (w_nt = 0) accumulating onto y, bias + relu, and the bf16 path against
torch's bf16-operand product."""
import pytest
import torch

from tests.gpu_util import assert_close

pytestmark = pytest.mark.gpu


def _rows(t, T, sB, sT, off=0):
    from mep_amd._lib import Rows
    return Rows(ptr=t.data_ptr() + t.element_size() * off, sB=sB, sT=sT, T=T)


def _launch(descs, dev, prec=0):
    """the chunked form (TGEMM_MIN_K lowered so every K runs on it)"""
    from mep_amd import _lib
    arr = _lib.DescArray(_lib.GemmDesc, descs, dev)
    min_k, _lib.TGEMM_MIN_K = _lib.TGEMM_MIN_K, 0
    try:
        assert _lib.tgemm_ok(arr.items)
    finally:
        _lib.TGEMM_MIN_K = min_k
    flags = prec | (0 if descs[0].w_nt else _lib.TGEMM_WT)
    _lib.call('mep_tgemm', arr.ptr, arr.n, max(d.ntok for d in descs), max(d.N for d in descs), flags)
    torch.cuda.synchronize()
    return arr


# three bf16 parts on both operands (fp32-level): rtol 1e-5, atol 1e-6 of max|y|
TOL = dict(rtol=1e-5, atol_frac=1e-6)


def _gd(x, y, w, ntok, N, K, ldw, w_nt=1, bias=None, table=None, accumulate=0, relu=0, alpha=1.0, bf16=0, ldt=0):
    from mep_amd._lib import GemmDesc
    return GemmDesc(x=x, y=y, w=w.data_ptr(), bias=bias.data_ptr() if bias is not None else 0,
                    table=table.data_ptr() if table is not None else 0, ntok=ntok, N=N, K=K, ldw=ldw, w_nt=w_nt,
                    accumulate=accumulate, relu=relu, alpha=alpha, bf16=bf16, ldt=ldt)


@pytest.mark.parametrize('N,Ks,B,T', [
    (96, (300, 35, 74), 64, 50),     # cmu-mosei cfg3: both slots, all three modalities in one launch
    (128, (768, 640, 205), 4, 300),  # Ren-MME cfg5 widths
    (32, (300, 35, 74), 3, 7),       # ragged: 21 tokens
    (64, (17,), 5, 1),               # T = 1 rows, K < 32
])
def test_tgemm_unify_vs_float64(N, Ks, B, T, cuda):
    torch.manual_seed(N + B + T)
    xs = [torch.randn(B, 2, T, K, device=cuda) for K in Ks]
    ws = [torch.randn(N, K, device=cuda) / K ** 0.5 for K in Ks]
    ys = [[torch.full((B, T, N), float('nan'), device=cuda) for _ in range(2)] for _ in Ks]
    descs = []
    for i, (x, w) in enumerate(zip(xs, ws)):
        K = x.shape[-1]
        for e in range(2):
            descs.append(_gd(_rows(x, T, 2 * T * K, K, e * T * K), _rows(ys[i][e], T, T * N, N), w, B * T, N, K, K))
    keep = _launch(descs, cuda)
    for i, (x, w) in enumerate(zip(xs, ws)):
        for e in range(2):
            want = x[:, e].double() @ w.double().t()
            assert_close(ys[i][e], want, name='K%d slot%d' % (x.shape[-1], e), **TOL)
    del keep


def test_tgemm_table_bias_relu_and_wide_n(cuda):
    """Conv1d unify + position table; N = 192 ([W_k; W_v], two N tiles) with bias and relu."""
    torch.manual_seed(11)
    B, T, K = 8, 50, 300
    x = torch.randn(B * T, K, device=cuda)
    w = torch.randn(96, K, device=cuda) / K ** 0.5
    tab = torch.randn(T, 96, device=cuda)
    y = torch.empty(B * T, 96, device=cuda)
    keep = _launch([_gd(_rows(x, T, T * K, K), _rows(y, T, T * 96, 96), w, B * T, 96, K, K, table=tab)], cuda)
    want = (x.double() @ w.double().t()).view(B, T, 96) + tab.double()
    assert_close(y.view(B, T, 96), want, name='table', **TOL)
    w2 = torch.randn(192, 96, device=cuda) / 96 ** 0.5
    b2 = torch.randn(192, device=cuda)
    y2 = torch.empty(B * T, 192, device=cuda)
    keep2 = _launch([_gd(_rows(y, T, T * 96, 96), _rows(y2, T, T * 192, 192), w2, B * T, 192, 96, 96, bias=b2,
                         relu=1)], cuda)
    want2 = torch.relu(y.double() @ w2.double().t() + b2.double())
    assert_close(y2, want2, name='N192 bias relu', **TOL)
    del keep, keep2


def test_tgemm_transposed_weight_accumulate(cuda):
    """dq_in += dQ W_q (W stored [K][N], w_nt = 0) and dkv_in = [dK | dV] [W_k; W_v] (K = 2D)."""
    torch.manual_seed(12)
    n, D = 3200, 96
    dq = torch.randn(n, D, device=cuda)
    wq = torch.randn(D, D, device=cuda) / D ** 0.5
    base = torch.randn(n, D, device=cuda)
    y = base.clone()
    dkv = torch.randn(n, 2 * D, device=cuda)
    wkv = torch.randn(2 * D, D, device=cuda) / D ** 0.5
    y2 = torch.empty(n, D, device=cuda)
    keep = _launch([_gd(_rows(dq, 50, 50 * D, D), _rows(y, 50, 50 * D, D), wq, n, D, D, D, w_nt=0, accumulate=1),
                    _gd(_rows(dkv, 50, 100 * D, 2 * D), _rows(y2, 50, 50 * D, D), wkv, n, D, 2 * D, D, w_nt=0)], cuda)
    assert_close(y, base.double() + dq.double() @ wq.double(), name='accumulate', **TOL)
    assert_close(y2, dkv.double() @ wkv.double(), name='K=2D', **TOL)
    del keep


@pytest.mark.parametrize('K', [768, 300])
def test_tgemm_bf16_path(K, cuda):
    """MEP_PREC_BF16: bf16 X and Y rows (MEP_BF16_STORE), plain bf16 operands, fp32 accumulation
    rounded to bf16 once on the store -- torch's bf16-operand product rounded to bf16."""
    from mep_amd import _lib
    torch.manual_seed(13)
    B, T, N = 4, 300, 96
    x = torch.randn(B * T, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda) / K ** 0.5
    y = torch.empty(B * T, N, device=cuda, dtype=torch.bfloat16)
    keep = _launch([_gd(_rows(x, T, T * K, K), _rows(y, T, T * N, N), w, B * T, N, K, K,
                        bf16=_lib.BF16_OPS | _lib.BF16_STORE)], cuda, prec=_lib.PREC_BF16)
    want = x.double() @ w.bfloat16().double().t()
    # one bf16 rounding of the output (2^-9 relative) on top of fp32 accumulation
    assert_close(y, want, rtol=4e-3, atol_frac=1e-4, name="bf16")
    assert torch.equal(y, y.float().bfloat16())
    del keep


def _launch_flags(descs, dev, flags):
    from mep_amd import _lib
    arr = _lib.DescArray(_lib.GemmDesc, descs, dev)
    _lib.call('mep_tgemm', arr.ptr, arr.n, max(d.ntok for d in descs), max(d.N for d in descs), flags)
    torch.cuda.synchronize()
    return arr


@pytest.mark.parametrize('bf', [True, False], ids=['bf16', 'fp32'])
@pytest.mark.parametrize('N,Ks,B,T,extra', [
    (128, (768, 640, 205), 4, 300, False),   # Ren-MME cfg5 unify widths (K = 205: a K tail, unaligned rows)
    (128, (768, 640, 35), 3, 7, True),       # ragged: 21 tokens; bias + position table + accumulate
    (96, (320, 64, 74), 5, 50, False),       # N tile 96 (6 column tiles)
    (256, (512,), 2, 130, True),             # two N tiles; 260 tokens (a partial last workgroup)
    (144, (768, 205), 3, 40, False),         # N % 32 = 16: waves whose weight rows end inside / past N
    (176, (640,), 2, 33, True),              # (every wave still issues its full DMA count per chunk)
])
def test_tgemm_dma_matches_register_staging(N, Ks, B, T, extra, bf, cuda):
    """MEP_TGEMM_DMA (weight ring by LDS-DMA) against the register-staged kernel on the same
    descriptors -- the same operands (one bf16 part, or three on the fp32 path), MFMAs and order:
    bit-identical -- and against torch's product (bf16 operands; float64 on the fp32 path); K tails
    and unaligned weight / X rows (K = 205, 35, 74) take the plain-load units of the same kernel."""
    from mep_amd import _lib
    torch.manual_seed(N + B + T)
    dt = torch.bfloat16 if bf else torch.float32
    xs = [torch.randn(B, 2, T, K, device=cuda).to(dt) for K in Ks]
    ws = [torch.randn(N, K, device=cuda) / K ** 0.5 for K in Ks]
    bias = torch.randn(N, device=cuda) if extra else None
    tab = torch.randn(T, N, device=cuda) if extra else None
    base = [[torch.randn(B, T, N, device=cuda).to(dt) if extra else
             torch.full((B, T, N), float('nan'), device=cuda).to(dt) for _ in range(2)] for _ in Ks]
    outs = {}
    for dma in (False, True):
        ys = [[b.clone() for b in bb] for bb in base]
        descs = []
        for i, (x, w) in enumerate(zip(xs, ws)):
            K = x.shape[-1]
            for e in range(2):
                descs.append(_gd(_rows(x, T, 2 * T * K, K, e * T * K), _rows(ys[i][e], T, T * N, N), w, B * T, N, K, K,
                                 bias=bias, table=tab, accumulate=int(extra),
                                 bf16=(_lib.BF16_OPS | _lib.BF16_STORE) if bf else 0))
        assert _lib.tgemm_dma_ok(descs)
        keep = _launch_flags(descs, cuda, (_lib.PREC_BF16 if bf else 0) | (_lib.TGEMM_DMA if dma else 0))
        outs[dma] = ys
        del keep
    for i, (x, w) in enumerate(zip(xs, ws)):
        for e in range(2):
            assert torch.equal(outs[True][i][e], outs[False][i][e]), (i, e)
            want = x[:, e].double() @ (w.bfloat16() if bf else w).double().t()
            if extra:
                want = want + bias.double() + tab.double() + base[i][e].double()
            tol = dict(rtol=4e-3, atol_frac=1e-4) if bf else dict(rtol=1e-5, atol_frac=1e-6)
            assert_close(outs[True][i][e], want, name='K%d slot%d' % (x.shape[-1], e), **tol)

