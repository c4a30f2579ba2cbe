"""mep_wgrad (csrc/gemm.hip k_wgrad + k_wgrad_reduce) against a torch fp32 statement of the same
weight gradients, dW_i = A^T B_i, on the row-view shapes the plans use and on the edge cases the
kernel's tiling has to handle: N and K not multiples of 32, several B operands concatenated on K,
strided slot views ([B, 2, T, d] slices), T = 1 views, odd token counts, chunks shorter than a
wave's token quarter, transposed output."""
import pytest
import torch

from tests.gpu_util import assert_close

pytestmark = pytest.mark.gpu


def _rows(t, T, sB, sT, off=0):
    from mep_amd._lib import Rows
    return Rows(ptr=t.data_ptr() + t.element_size() * off, sB=sB, sT=sT, T=T)


def _run(items, dev, tok_per_split=None, bf16=False):
    from mep_amd import trimodal
    from mep_amd._lib import launch
    ws, arr, n_wg, rmax = trimodal.make_wgrad(items, dev, tok_per_split=tok_per_split, bf16=bf16)
    launch('mep_wgrad', arr, n_wg)
    launch('mep_wgrad_reduce', arr, rmax)
    torch.cuda.synchronize()
    return ws, arr


CASES = [
    # (N, [K_i], B, T)
    (96, [96], 64, 50),          # cmu proj.weight
    (96, [96, 96], 64, 50),      # cmu minus.weight = dZ^T [q | xp]
    (96, [300], 64, 50),         # unify linguistic
    (96, [35], 64, 50),          # unify visual (K % 4 != 0)
    (96, [74], 64, 50),          # unify acoustic
    (128, [128, 128], 4, 300),   # Ren-MME minus.weight
    (80, [40], 3, 7),            # N, K off the 32 grid, odd token count (21)
    (32, [64, 32, 7], 5, 13),    # three operands, last one ragged
    (64, [200], 9, 1),           # T = 1 views (head-style rows)
    (14, [7], 1, 5),             # a handful of tokens: most waves idle
]


@pytest.mark.parametrize('N,Ks,B,T', CASES)
def test_wgrad_vs_torch(N, Ks, B, T, cuda):
    torch.manual_seed(N * 1000 + sum(Ks) + B * 7 + T)
    n = B * T
    A = torch.randn(B, T, N, device=cuda)
    # B operands as slot 1 of a [B, 2, T, K] tensor: a strided view like the plans' input slots
    Bs = [torch.randn(B, 2, T, K, device=cuda) for K in Ks]
    outs = [torch.full((N, K), float('nan'), device=cuda) for K in Ks]
    item = (_rows(A, T, T * N, N), N, n,
            [(_rows(b, T, 2 * T * K, K, T * K), K, o.data_ptr(), K) for b, K, o in zip(Bs, Ks, outs)])
    keep = _run([item], cuda)
    a2 = A.reshape(n, N).double()
    for b, K, o in zip(Bs, Ks, outs):
        want = a2.t() @ b[:, 1].reshape(n, K).double()
        assert_close(o, want, rtol=1e-5, atol_frac=1e-6, name='N%d K%d' % (N, K))
    del keep


@pytest.mark.parametrize('N,Ks,B,T', [CASES[1], CASES[3], CASES[5], CASES[7], CASES[8], CASES[6]])
def test_wgrad_bf16_vs_torch(N, Ks, B, T, cuda):
    """bf16 path: bf16 operand rows (include/mep.h MEP_BF16_STORE), read as column-pair dwords --
    4-byte aligned, token-linear rows (odd widths padded to even, as the plans pad the features) --
    and exactly the products of the bf16 values (each exact in fp32), summed in fp32: checked
    against float64 sums."""
    torch.manual_seed(N * 1000 + sum(Ks) + B * 7 + T + 1)
    n = B * T
    A = torch.randn(B, T, N, device=cuda).bfloat16()
    Kp = [K + K % 2 for K in Ks]
    Bs = [torch.randn(B, T, k, device=cuda).bfloat16() for k in Kp]
    outs = [torch.full((N, K), float('nan'), device=cuda) for K in Ks]
    item = (_rows(A, T, T * N, N), N, n,
            [(_rows(b, T, T * k, k), K, o.data_ptr(), K) for b, k, K, o in zip(Bs, Kp, Ks, outs)])
    keep = _run([item], cuda, bf16=True)
    a2 = A.reshape(n, N).double()
    for b, K, o in zip(Bs, Ks, outs):
        want = a2.t() @ b.reshape(n, -1)[:, :K].double()
        assert_close(o, want, rtol=1e-5, atol_frac=1e-6, name='bf16 N%d K%d' % (N, K))
    del keep


@pytest.mark.parametrize('tps', [8, 24, 64, 1000])
def test_wgrad_fixed_splits_and_transposed_out(tps, cuda):
    """Fixed token chunks (split boundaries inside batch rows, a chunk shorter than 4 waves x 2
    tokens) and out_trans (dW written [K][N])."""
    torch.manual_seed(tps)
    B, T, N, K = 6, 17, 96, 160
    n = B * T
    A = torch.randn(n, N, device=cuda)
    X = torch.randn(n, K, device=cuda)
    out = torch.full((K, N), float('nan'), device=cuda)
    item = (_rows(A, T, T * N, N), N, n, [(_rows(X, T, T * K, K), K, out.data_ptr(), N)], 1)
    keep = _run([item], cuda, tok_per_split=tps)
    want = (A.double().t() @ X.double()).t()
    assert_close(out, want, rtol=1e-5, atol_frac=1e-6, name='tps%d' % tps)
    del keep


def test_wgrad_many_items_one_launch(cuda):
    """The bench plan's shape of launch: many items of different geometry in one flat grid."""
    torch.manual_seed(1)
    B, T = 64, 50
    n = B * T
    items, checks = [], []
    for N, Ks in [(96, [96])] * 5 + [(96, [96, 96])] * 5 + [(96, [300]), (96, [35]), (96, [74])]:
        A = torch.randn(n, N, device=cuda)
        Xs = [torch.randn(n, K, device=cuda) for K in Ks]
        outs = [torch.empty(N, K, device=cuda) for K in Ks]
        items.append((_rows(A, T, T * N, N), N, n,
                      [(_rows(x, T, T * K, K), K, o.data_ptr(), K) for x, K, o in zip(Xs, Ks, outs)]))
        checks.append((A, Xs, outs))
    keep = _run(items, cuda)
    for A, Xs, outs in checks:
        for x, o in zip(Xs, outs):
            assert_close(o, A.double().t() @ x.double(), rtol=1e-5, atol_frac=1e-6, name='multi')
    del keep
