"""Evaluation / threshold sweep: host metric logic and the oracle on the
CPU; mep_threshold_sweep and the rf_test / cmu_test drivers against the oracle on the GPU.

Parity bar: confusion counts bit-exact (integer work); F1 / accuracy within 1e-12 of sklearn's
(float64 arithmetic in a different order); selected thresholds identical."""
import numpy as np
import pytest
import torch
from sklearn.metrics import accuracy_score, f1_score

from mep_amd import evaluate
from oracle import evaluate as oev


def _counts_from_lists(y, p):
    y, p = np.asarray(y), np.asarray(p)
    return np.array([(y & p).sum(), (~y & p).sum(), (y & ~p).sum(), (~y & ~p).sum()]) if y.dtype == bool else \
        _counts_from_lists(y != 0, p != 0)


@pytest.mark.parametrize('case', ['random', 'all_neg', 'all_pos', 'pred_all_pos', 'pred_all_neg', 'one'])
def test_metrics_match_sklearn(case):
    rng = np.random.default_rng(7)
    n = 1 if case == 'one' else 257
    y = rng.random(n) < 0.3
    p = rng.random(n) < 0.5
    if case == 'all_neg':
        y[:] = False
    if case == 'all_pos':
        y[:] = True
    if case == 'pred_all_pos':
        p[:] = True
    if case == 'pred_all_neg':
        p[:] = False
    f1, acc = evaluate.metrics_from_counts(_counts_from_lists(y, p))
    yl, pl = y.astype(int).tolist(), p.astype(int).tolist()
    assert abs(float(f1) - f1_score(yl, pl, average='weighted', zero_division=0)) < 1e-12
    assert abs(float(acc) - accuracy_score(yl, pl)) < 1e-12


def _rf_batches(seed, shapes):
    g = torch.Generator().manual_seed(seed)
    out = []
    for B, P in shapes:
        p1 = torch.randn(B, P, 6, generator=g)
        p2 = torch.randn(B, P, 6, generator=g)
        lab = (torch.rand(B, P, 6, generator=g) < 0.3).long()
        lens = torch.randint(0, P + 1, (B,), generator=g)
        mask = (torch.arange(P)[None, :] < lens[:, None]).long()
        mask[0, -1] = 1                       # a 1 after a 0: the walk stops at the first 0
        out.append((p1, p2, lab, mask))
    return out


def _rf_counts_oracle(batches, n_thr):
    tot = 0
    for p1, p2, lab, mask in batches:
        c, _ = oev.sweep_counts([p1.reshape(-1, 6).numpy(), p2.reshape(-1, 6).numpy()], (0.6, 0.4),
                                lab.reshape(-1, 6).numpy(), oev.rf_thresholds(n_thr), row_mask=mask.numpy())
        tot = tot + c
    return tot


def test_rf_counts_path_matches_reference_loop():
    """The counts formulation (per-threshold counts, prefix sum, metrics from counts, strict > pick)
    reproduces the reference's list-appending loop, accumulation across thresholds included."""
    n_thr = 400
    batches = _rf_batches(3, [(3, 6), (2, 6)])
    want = oev.rf_test(batches, n_thr)
    got = evaluate.rf_select(_rf_counts_oracle(batches, n_thr), n_thr, cumulative=True)
    assert len(got) == 18
    for k in range(6):
        assert got[3 * k + 2] == want[3 * k + 2], (k, got, want)
        assert abs(got[3 * k] - want[3 * k]) < 1e-12 and abs(got[3 * k + 1] - want[3 * k + 1]) < 1e-12


def test_cmu_counts_path_matches_reference_loop():
    g = torch.Generator().manual_seed(5)
    rows = [([torch.randn(1, 7, generator=g) * 0.5 for _ in range(4)], (torch.rand(1, 7, generator=g) < 0.3).long())
            for _ in range(97)]
    want = oev.cmu_test(rows)
    thr = np.zeros((1, 7), np.float32)
    for _, c, t in oev.CMU_CLASSES:
        thr[0, c] = t
    cnt, _ = oev.sweep_counts([torch.cat([r[0][m] for r in rows]).numpy() for m in range(4)], [1.0] * 4,
                              torch.cat([r[1] for r in rows]).numpy(), thr, post_div=4.0, per_class=True)
    f1, acc = evaluate.metrics_from_counts(cnt)
    for k, c, _ in oev.CMU_CLASSES:
        assert abs(acc[0, c] - want[k][0]) < 1e-12 and abs(f1[0, c] - want[k][1]) < 1e-12, k


def _eval_golden():
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'eval_golden.npz'))
    return {k: z[k] for k in z.files}


def test_rf_oracle_pinned_to_reference_test_loop():
    """oracle/evaluate.rf_test against the reference's own test() (others/realformer.py:395-477,
    AST-extracted and run on recorded scores by tests/golden/make_eval_golden.py), cumulative lists
    and strict '>' selection included; then the repo's counts formulation against the same."""
    g = _eval_golden()
    batches = [(torch.from_numpy(g['rf_pred1'][k]), torch.from_numpy(g['rf_pred2'][k]),
                torch.from_numpy(g['rf_label'][k]), torch.from_numpy(g['rf_mask'][k]))
               for k in range(g['rf_pred1'].shape[0])]
    want = g['rf_best']
    got = oev.rf_test(batches, 400)
    np.testing.assert_allclose(np.array(got, np.float64), want, rtol=0, atol=1e-12)
    got2 = evaluate.rf_select(_rf_counts_oracle(batches, 400), 400, cumulative=True)
    np.testing.assert_allclose(np.array(got2, np.float64), want, rtol=0, atol=1e-12)


def test_cmu_oracle_pinned_to_reference_test_loop():
    """oracle/evaluate.cmu_test against the accuracy / F1 lines the reference's test()
    (cmu-mosei/run.py:456-498) printed for the recorded 4-model scores."""
    g = _eval_golden()
    preds, labels = g['cmu_preds'], g['cmu_label']
    rows = [([torch.from_numpy(preds[m, k]) for m in range(preds.shape[0])], torch.from_numpy(labels[k][None]))
            for k in range(labels.shape[0])]
    got = oev.cmu_test(rows)
    for i, k in enumerate(('happ', 'sadn', 'ange', 'fear', 'disg', 'surp')):
        np.testing.assert_allclose(got[k], g['cmu_metrics'][i], rtol=0, atol=1e-12, err_msg=k)


# ------------------------------------------------------------------------------------------ GPU
SWEEP_CASES = [
    # (N, C, n_thr, n_models, P, per_class, strided)
    (1, 6, 1, 1, 0, False, False),
    (257, 6, 400, 2, 0, False, False),
    (300, 6, 65, 2, 6, False, True),
    (511, 7, 1, 4, 0, True, False),
    (64, 16, 130, 8, 4, True, False),
    (0, 6, 10, 2, 0, False, False),
    (1000, 9, 63, 3, 0, False, False),
]


@pytest.mark.gpu
@pytest.mark.parametrize('case', SWEEP_CASES)
def test_sweep_counts_gpu(cuda, case):
    N, C, n_thr, M, P, per_class, strided = case
    rng = np.random.default_rng(N * 31 + C)
    if strided:
        base = [rng.standard_normal((N, C + 3)).astype(np.float32) for _ in range(M)]
        preds_np = [b[:, :C] for b in base]
        preds = [torch.from_numpy(b).to(cuda)[:, :C] for b in base]
    else:
        preds_np = [rng.standard_normal((N, C)).astype(np.float32) for _ in range(M)]
        preds = [torch.from_numpy(p).to(cuda) for p in preds_np]
    if N > 2:
        preds_np[0][1, 0] = np.nan           # NaN scores predict 0 (torch.where(pred > t))
        preds[0][1, 0] = float('nan')
    labels = (rng.random((N, C)) < 0.3).astype(np.int64) * rng.integers(1, 3, (N, C))
    weights = rng.uniform(0.1, 1.0, M).astype(np.float32).tolist()
    thr = rng.uniform(-2, 2, (n_thr, C) if per_class else n_thr).astype(np.float32)
    mask = None
    if P:
        lens = rng.integers(0, P + 1, N // P)
        mask = (np.arange(P)[None, :] < lens[:, None]).astype(np.int64)
        mask[:, -1] = 1
    want, want_s = oev.sweep_counts(preds_np, weights, labels, thr, post_div=float(M), row_mask=mask,
                                    per_class=per_class)
    scores = torch.empty(N, C, device=cuda)
    got = evaluate.threshold_sweep(preds, torch.from_numpy(labels).to(cuda), torch.from_numpy(thr).to(cuda),
                                   weights=weights, post_div=float(M),
                                   row_mask=None if mask is None else torch.from_numpy(mask).to(cuda),
                                   scores=scores)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().astype(np.int64), want)
    np.testing.assert_array_equal(scores.cpu().numpy(), want_s)   # bit-exact fp32 combine


SORTED_CASES = [
    # (N, C, n_thr, n_models, P, per_class)
    (24576, 6, 400, 2, 6, False),     # realformer shape
    (3000, 7, 1, 4, 0, True),         # cmu: per-class fixed thresholds
    (513, 16, 300, 3, 0, True),
    (5000, 1, 2000, 1, 0, False),     # many thresholds: several bins per lane in the suffix pass
]


@pytest.mark.gpu
@pytest.mark.parametrize('case', SORTED_CASES)
def test_sweep_sorted_path_gpu(cuda, case):
    """Histogram + suffix-sum formulation (sorted thresholds, ties, NaN scores, scores equal to a
    threshold) against the oracle and against the direct-compare kernel."""
    N, C, n_thr, M, P, per_class = case
    rng = np.random.default_rng(N + C + n_thr)
    preds_np = [np.round(rng.standard_normal((N, C)), 2).astype(np.float32) for _ in range(M)]
    preds_np[0][::97, 0] = np.nan
    labels = (rng.random((N, C)) < 0.3).astype(np.int64)
    base = np.sort(np.round(rng.uniform(-2, 2, (n_thr, C) if per_class else n_thr), 2).astype(np.float32), axis=0)
    if n_thr > 3:
        base[1] = base[2]                                        # a tie
    mask = None
    if P:
        lens = rng.integers(0, P + 1, N // P)
        mask = (np.arange(P)[None, :] < lens[:, None]).astype(np.int64)
    want, want_s = oev.sweep_counts(preds_np, [1.0] * M, labels, base, post_div=float(M), row_mask=mask,
                                    per_class=per_class)
    preds = [torch.from_numpy(p).to(cuda) for p in preds_np]
    lab = torch.from_numpy(labels).to(cuda)
    thr = torch.from_numpy(base).to(cuda)
    mk = None if mask is None else torch.from_numpy(mask).to(cuda)
    scores = torch.empty(N, C, device=cuda)
    got = evaluate.threshold_sweep(preds, lab, thr, post_div=float(M), row_mask=mk, scores=scores, sorted_path=True)
    direct = evaluate.threshold_sweep(preds, lab, thr, post_div=float(M), row_mask=mk, sorted_path=False)
    again = evaluate.threshold_sweep(preds, lab, thr, post_div=float(M), row_mask=mk, sorted_path=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().astype(np.int64), want)
    np.testing.assert_array_equal(direct.cpu().numpy(), got.cpu().numpy())
    np.testing.assert_array_equal(again.cpu().numpy(), got.cpu().numpy())   # workspace left zeroed
    np.testing.assert_array_equal(scores.cpu().numpy(), want_s)


@pytest.mark.gpu
def test_sweep_accumulates_across_calls(cuda):
    rng = np.random.default_rng(11)
    thr = torch.from_numpy(evaluate.rf_thresholds(400)).to(cuda)
    counts, want = None, 0
    for _ in range(3):
        p = rng.standard_normal((96, 6)).astype(np.float32)
        lab = (rng.random((96, 6)) < 0.3).astype(np.int64)
        counts = evaluate.threshold_sweep([torch.from_numpy(p).to(cuda)], torch.from_numpy(lab).to(cuda), thr,
                                          counts=counts)
        want = want + oev.sweep_counts([p], [1.0], lab, evaluate.rf_thresholds(400))[0]
    np.testing.assert_array_equal(counts.cpu().numpy().astype(np.int64), want)


def _rows(tensors):
    """Tensors in data_loader column order -> the list of per-utterance tuples it yields."""
    return list(zip(*[t.numpy() for t in tensors]))


def _perturbed(models):
    with torch.no_grad():
        for i, m in enumerate(models):
            for p in m.parameters():
                p.mul_(1.0 - 0.07 * i)
    return models


@pytest.mark.gpu
def test_rf_test_models_gpu(cuda):
    """realformer test(model_1, model_2) end to end: two State_Transfer models on the HIP plan, the
    sweep on the GPU; the oracle runs the reference loop (realformer.py:395-477) on the same logits."""
    from mep_amd import realformer as rf
    from tests.golden import fixtures
    from tests.test_gpu_realformer import _state
    meta, _ = fixtures.load('rf_state_small')
    models = _perturbed([_state(meta, cuda), _state(meta, cuda)])
    cols = fixtures.batch(meta)
    cols2 = [c.flip(0) if c.dtype == torch.float32 else c for c in cols]   # a second batch
    batches = [_rows(cols), _rows(cols2)]
    got = evaluate.rf_test(models[0], models[1], batches, n_thr=400, device=cuda)
    ref_in = []
    with torch.no_grad():
        for b in batches:
            l, v, a, label, lm, vm, am, mask = rf._to_device(b, cuda)
            ref_in.append((models[0](l, v, a, lm, vm, am).cpu(), models[1](l, v, a, lm, vm, am).cpu(),
                           label.cpu(), mask.cpu()))
    want = oev.rf_test(ref_in, 400)
    for k in range(6):
        assert got[3 * k + 2] == want[3 * k + 2], (k, got, want)
        assert abs(got[3 * k] - want[3 * k]) < 1e-12 and abs(got[3 * k + 1] - want[3 * k + 1]) < 1e-12


@pytest.mark.gpu
def test_cmu_test_models_gpu(cuda):
    """cmu-mosei test(model_1..model_4) (run.py:456-498): four Concat_Trans models on the HIP plan,
    batched; the oracle runs the reference's batch-1 loop on the same per-row logits."""
    from mep_amd import cmu_mosei
    from tests.golden import fixtures
    from tests.gpu_util import cmu_model
    meta, _ = fixtures.load('cmu_small')
    models = _perturbed([cmu_model(meta, cuda) for _ in range(4)])
    cols = fixtures.batch(meta)
    batches = [_rows(cols)]
    got = evaluate.cmu_test(models, batches, device=cuda, verbose=False)
    l, v, a, lm, vm, am, label = cmu_mosei._to_device(batches[0], cuda)
    with torch.no_grad():
        outs = [m(l, v, a, lm, vm, am).cpu() for m in models]
    rows = [([o[i:i + 1] for o in outs], label[i:i + 1].cpu()) for i in range(label.shape[0])]
    want = oev.cmu_test(rows)
    for k in want:
        assert abs(got[k][0] - want[k][0]) < 1e-12 and abs(got[k][1] - want[k][1]) < 1e-12, k
