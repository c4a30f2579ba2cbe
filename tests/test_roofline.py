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


def test_valu_floor_names_the_limiter():
    # 12e6 wave64 VALU instructions: 4 cycles each over 1024 SIMDs at 2.4 GHz = 19.5 us, beside a
    # 16-us HBM floor (128 MB) -> VALU-limited, while the contract's bound stays hbm
    e = rl.roofline_entry('mep_attn_bwd', flops=1e9, nbytes=128e6, seconds=38e-6, valu=(12e6, 'test'))
    assert e['bound'] == 'hbm' and e['limiter'] == 'valu'
    assert e['valu']['floor_us'] == pytest.approx(4 * 12e6 / (1024 * 2.4e9) * 1e6, rel=1e-3)
    e = rl.roofline_entry('mep_attn_bwd', flops=1e9, nbytes=128e6, seconds=38e-6, valu=(1e6, 'test'))
    assert e['limiter'] == 'hbm'


def test_attention_bytes_count_shared_inputs_once():
    """cmu-mosei cfg3: each of the 6 unified feature tensors (2 encoders x 3 modalities) is the
    query of 3 blocks and the key / value of 3: the attention launches read it once"""
    from mep_amd import cmu_mosei
    B, T, D, H = 64, 50, 96, 6
    m = cmu_mosei.Concat_Trans(dim=D, l_len=T, v_len=T, a_len=T, n_heads=H, n_layers=1, ffn=1)
    plan = m.mep_runner('cpu').plan(B, (T, T, T))
    costs = rl.launch_costs(plan)
    u = 4 * B * T * D
    fwd = 6 * u + 18 * (u + 8 * B * H * T) + 6 * 4 * B * T           # U once, X + stats per block, masks
    assert costs['mep_attn_fwd'][1] == fwd
    bwd = 6 * u + 18 * (4 * u + u + 8 * B * H * T) + 6 * 4 * B * T   # + x, dx, dq r+w, dkv per block
    assert costs['mep_attn_bwd'][1] == bwd
    assert costs['mep_attn_fwd'][0] == 18 * B * 4 * T * T * D
