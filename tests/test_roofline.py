"""Roofline pricing (mep_amd/roofline.py): the compute peaks follow the bf16 products per fp32
product of each kernel's arithmetic."""
import pytest

from mep_amd import roofline as rl


def test_compute_peaks_follow_product_counts():
    bf = rl.BF16_PEAK
    assert rl.compute_peak('mep_wgrad') == pytest.approx(bf / 6)
    assert rl.compute_peak('mep_attn_fwd') == pytest.approx(bf / 6)          # 3-part scores and P.V
    assert rl.compute_peak('mep_attn_bwd') == pytest.approx(bf / 3.8)        # (4+4+4+4+3) / 5 products
    assert rl.compute_peak('mep_block_epi_fwd', 96) == pytest.approx(bf / 6)
    assert rl.compute_peak('mep_block_epi_fwd', 128) == pytest.approx(bf / 5)
    assert rl.compute_peak('mep_block_epi_bwd', 128) == pytest.approx(bf / 5)
    assert bf / 6 < rl.compute_peak('mep_block_epi_bwd', 96) < bf / 5
    assert rl.compute_peak('mep_gemm') == rl.F32_PEAK
    assert rl.compute_peak('mep_attn_bwd', bf16=True) == bf


def test_roofline_entry_picks_the_binding_side():
    e = rl.roofline_entry('mep_attn_bwd', flops=1e9, nbytes=1e9, seconds=1e-3)
    assert e['bound'] == 'hbm' and e['frac'] == pytest.approx(1e9 / 1e-3 / rl.HBM_PEAK, rel=1e-3)
    e = rl.roofline_entry('mep_wgrad', flops=1e12, nbytes=1e6, seconds=1e-2)
    assert e['bound'] == 'mfma' and e['peak'] == pytest.approx(rl.BF16_PEAK / 6 / 1e12, rel=1e-3)
