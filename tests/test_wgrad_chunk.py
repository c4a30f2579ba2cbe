"""Weight-gradient segment length (trimodal.wgrad_chunk) on the bench plans, CPU only: the bf16
instance picks the round count with the least modelled time, the fp32 instance one round."""
import pytest

from mep_amd import cmu_mosei, ren_mme, trimodal


def _items(m, B, T, bf16):
    p = m.mep_runner('cpu').plan(B, T, bf16=bf16)
    return [tuple(it) + (0,) * (5 - len(it)) for it in p._wgrad_items]


@pytest.mark.parametrize('bf16', [True, False])
def test_wgrad_chunk_rounds(bf16, monkeypatch):
    monkeypatch.setattr(trimodal, 'WG_BALANCE', False)   # the uniform-chunk form (MEP_WG_BALANCE=0)
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


def _worst(items, segs, bf16):
    """the costliest segment, tokens x (MT + KT tiles of its column group)"""
    geo = {}
    for i, (_, N, _, bs, _) in enumerate(items):
        K = sum(b[1] for b in bs)
        mt, kt, _ = trimodal.wgrad_geometry(N, K, bf16)
        geo[i] = (mt, kt, trimodal.cdiv(K, 32))
    out = 0
    for s in segs:
        for (i, cg, t0, t1, _) in s:
            mt, kt, kts = geo[i]
            out = max(out, (t1 - t0) * (mt + min(kt, kts - cg * kt)))
    return out


@pytest.mark.parametrize('bf16', [True, False])
def test_wgrad_balanced_counts(bf16, monkeypatch):
    """trimodal.wgrad_counts: the launch fills whole rounds of workgroup slots (no slot left
    empty at cfg3), every unit is cut, and the costliest segment is no costlier than with one
    uniform chunk"""
    n = trimodal.wg_target(bf16)
    cfg3 = _items(cmu_mosei.Concat_Trans(96, 50, 50, 50, 6, 1, 1), 64, (50, 50, 50), bf16)
    cfg5 = _items(ren_mme.Base_model(dim=128, l_len=300, v_len=300, a_len=300, n_heads=8, n_layers=1), 32,
                  (300, 300, 300), bf16)
    for items in (cfg3, cfg5):
        units = trimodal._wgrad_units(items, bf16)
        cnt = trimodal.wgrad_counts(items, n, bf16)
        assert set(cnt) == {(i, cg) for (i, cg, _) in units} and all(k >= 1 for k in cnt.values())
        assert sum(cnt.values()) % n == 0 or sum(cnt.values()) == len(units)
        monkeypatch.setattr(trimodal, 'WG_BALANCE', True)
        bal = trimodal.wgrad_segments(items, n, bf16=bf16)[0]
        monkeypatch.setattr(trimodal, 'WG_BALANCE', False)
        uni = trimodal.wgrad_segments(items, n, bf16=bf16)[0]
        assert _worst(items, bal, bf16) <= _worst(items, uni, bf16)
        # every token of every unit in exactly one segment
        cover = {}
        for s in bal:
            for (i, cg, t0, t1, _) in s:
                cover.setdefault((i, cg), []).append((t0, t1))
        for (i, cg, nt) in units:
            spans = sorted(cover[(i, cg)])
            assert spans[0][0] == 0 and spans[-1][1] == nt and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert sum(trimodal.wgrad_counts(cfg3, n, bf16).values()) == n      # cfg3: every slot
