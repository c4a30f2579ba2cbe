"""mep_unify (csrc/gemm.hip k_unify) against a torch fp32 statement of Unify_Dimension's Linear
(cmu-mosei/run.py:210-214, Ren-MME/run.py:161-166) on the plans' input layout -- slot views of a
[B, 2, T, d] tensor -- including unaligned K (35, 74, 205: scalar X loads), the L2-resident
weight path (Ren-MME text, K = 768), ragged token counts and several problems in one launch."""
import pytest
import torch

from tests.gpu_util import assert_close

pytestmark = pytest.mark.gpu


def _desc(x, slot, w, y, table=None):
    from mep_amd._lib import GemmDesc, Rows
    B, E, T, K = x.shape
    N = w.shape[0]
    xr = Rows(ptr=x.data_ptr() + 4 * slot * T * K, sB=E * T * K, sT=K, T=T)
    yr = Rows(ptr=y.data_ptr(), sB=T * N, sT=N, T=T)
    return GemmDesc(x=xr, y=yr, w=w.data_ptr(), bias=0, table=table.data_ptr() if table is not None else 0,
                    ntok=B * T, N=N, K=K, ldw=K, w_nt=1, accumulate=0, relu=0, alpha=1.0)


def _run(descs, dev):
    from mep_amd import trimodal
    from mep_amd._lib import launch
    arr, n_wg = trimodal.make_unify(descs, dev)
    launch('mep_unify', arr, n_wg)
    torch.cuda.synchronize()
    return arr


@pytest.mark.parametrize('N,Ks,B,T', [
    (96, (300, 35, 74), 64, 50),     # cmu-mosei cfg3 (both slots, all three modalities)
    (128, (768, 640, 205), 4, 300),  # Ren-MME cfg5 shapes (text / video through L2)
    (32, (300, 35, 74), 3, 7),       # ragged: 21 tokens, one partial 16-token tile
    (64, (17,), 5, 1),               # T = 1 rows, K < 16
])
def test_unify_vs_torch(N, Ks, B, T, cuda):
    torch.manual_seed(N + B + T)
    xs = [torch.randn(B, 2, T, K, device=cuda) for K in Ks]
    ws = [torch.randn(N, K, device=cuda) / K ** 0.5 for K in Ks]
    ys = [[torch.full((B, T, N), float('nan'), device=cuda) for _ in range(2)] for _ in Ks]
    descs = [_desc(x, e, w, ys[i][e]) for i, (x, w) in enumerate(zip(xs, ws)) for e in range(2)]
    keep = _run(descs, cuda)
    for i, (x, w) in enumerate(zip(xs, ws)):
        for e in range(2):
            want = x[:, e].double() @ w.double().t()
            assert_close(ys[i][e], want, rtol=1e-5, atol_frac=1e-6, name='K%d slot%d' % (x.shape[-1], e))
    del keep


def test_unify_table(cuda):
    """table[t % T] added (the realformer Conv1d unify + position embedding form)."""
    torch.manual_seed(3)
    B, T, K, N = 6, 50, 300, 96
    x = torch.randn(B, 2, T, K, device=cuda)
    w = torch.randn(N, K, device=cuda) / K ** 0.5
    tab = torch.randn(T, N, device=cuda)
    y = torch.empty(B, T, N, device=cuda)
    keep = _run([_desc(x, 1, w, y, tab)], cuda)
    assert_close(y, x[:, 1].double() @ w.double().t() + tab.double(), rtol=1e-5, atol_frac=1e-6, name='table')
    del keep
