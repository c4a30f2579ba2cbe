"""MEP_TGEMM_DMA's host gate (_lib.tgemm_dma_ok, include/mep.h): no GPU needed."""
from mep_amd import _lib


def test_tgemm_dma_gate():
    """the bf16-path launches with every weight stored [N][K] (w_nt) take the LDS-DMA kernel"""
    R = _lib.Rows

    def gd(K, N, w_nt=1):
        return _lib.GemmDesc(x=R(ptr=4096, sB=0, sT=K, T=1), y=R(ptr=8192, sB=0, sT=N, T=1),
                             w=4096, ntok=16, N=N, K=K, ldw=K, w_nt=w_nt)
    assert _lib.tgemm_dma_ok([gd(768, 128), gd(640, 128), gd(205, 128)])
    assert not _lib.tgemm_dma_ok([gd(768, 128), gd(96, 96, w_nt=0)])
