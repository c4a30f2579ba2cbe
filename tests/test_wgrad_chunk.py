"""Weight-gradient segment length (trimodal.wgrad_chunk) on the bench plans, CPU only: the bf16
instance picks the round count with the least modelled time, the fp32 instance one round."""
import pytest

from mep_amd import cmu_mosei, ren_mme, trimodal


def _items(m, B, T, bf16):
    p = m.mep_runner('cpu').plan(B, T, bf16=bf16)
    return [tuple(it) + (0,) * (5 - len(it)) for it in p._wgrad_items]


@pytest.mark.parametrize('bf16', [True, False])
def test_wgrad_chunk_rounds(bf16):
    n = trimodal.wg_target(bf16)
    cfg3 = _items(cmu_mosei.Concat_Trans(96, 50, 50, 50, 6, 1, 1), 64, (50, 50, 50), bf16)
    cfg5 = _items(ren_mme.Base_model(dim=128, l_len=300, v_len=300, a_len=300, n_heads=8, n_layers=1), 32,
                  (300, 300, 300), bf16)
    for items in (cfg3, cfg5):
        ch = trimodal.wgrad_chunk(items, n, bf16=bf16)
        segs = trimodal.wgrad_segments(items, n, bf16=bf16)[0]
        assert ch % 8 == 0 and all(t1 - t0 <= ch for s in segs for (_, _, t0, t1, _) in s)
        one = trimodal._wgrad_fit(trimodal._wgrad_units(items, bf16), n)
        if not bf16:
            assert ch == one and len(segs) <= n          # one round of resident workgroups
    if bf16:
        assert trimodal.wgrad_chunk(cfg3, n, bf16=True) == 1072   # one round (210 workgroups)
        assert trimodal.wgrad_chunk(cfg5, n, bf16=True) == 3200   # two rounds (480), not 160 x 9,600
