"""Evaluation oracle: ensemble combine + threshold sweep (TEST INFRASTRUCTURE ONLY -- see
oracle/__init__.py).  SURVEY.md section 8(f) row 2.

A line-by-line restatement of the reference's test() loops over precomputed model scores, in
fp32 torch arithmetic with the reference's own metric calls (sklearn ``accuracy_score`` and
``f1_score(average='weighted')``, the third-party code the reference uses; sklearn 1.7.2 here).

Pinning: the reference ships no evaluation fixtures and its test() functions cannot run as
written (CUDA tensors, data on ``/home``).  tests/golden/make_eval_golden.py therefore runs the
reference's own test() loops (AST-extracted, CPU tensors for ``torch.cuda.*Tensor``, a data_loader
and score-returning models over recorded synthetic scores) and records their outputs
(tests/golden/eval_golden.npz); tests/test_eval.py pins ``rf_test`` and ``cmu_test`` to them.

Deliberately reproduced reference behaviour (others/realformer.py:404-477): the per-class label
and prediction lists are created once, outside the 400-threshold loop, so the metrics at
threshold t are computed over the predictions of every threshold 0..t (a cumulative sweep).
"""
import numpy as np
import torch
from sklearn.metrics import accuracy_score, f1_score

RF_CLASSES = ('happ', 'sadn', 'ange', 'surp', 'disg', 'fear')   # realformer.py:440-451 column order


def rf_thresholds(n_thr=400):
    """threshold = t/200 - 1.0 for t in range(400) (realformer.py:411-412), as the fp32 value the
    comparison ``pred > threshold`` uses (torch compares an fp32 tensor in fp32)."""
    return np.array([t / 200 - 1.0 for t in range(n_thr)], dtype=np.float32)


def rf_test(batches, n_thr=400):
    """others/realformer.py:395-477 over precomputed scores.

    batches: list of (pred_1 [B,P,6] fp32, pred_2 [B,P,6] fp32, label [B,P,6] int64,
    mask [B,P] int64) -- the per-batch model outputs the reference recomputes for every threshold
    (identical each time: the models are in eval mode under no_grad).
    Returns the reference's 18-tuple (best f1, its acc, its threshold per class)."""
    lists = {k: ([], []) for k in RF_CLASSES}
    best = {k: [0, 0, 0] for k in RF_CLASSES}
    for t in range(n_thr):
        threshold = t / 200 - 1.0
        for pred_1, pred_2, label, mask in batches:
            pred = pred_1 * 0.6 + pred_2 * 0.4                              # :420
            pred = torch.where(pred > threshold, torch.ones_like(pred), torch.zeros_like(pred))
            for i in range(len(mask)):
                for j in range(mask.shape[1]):
                    if int(mask[i][j]) == 1:                                # :425-437
                        for c, k in enumerate(RF_CLASSES):
                            lists[k][0].append(int(label[i][j][c]))
                            lists[k][1].append(int(pred[i][j][c]))
                    else:
                        break
        for k in RF_CLASSES:                                                # :438-473
            acc = accuracy_score(lists[k][0], lists[k][1])
            f1 = f1_score(lists[k][0], lists[k][1], average='weighted')
            if f1 > best[k][0]:
                best[k] = [f1, acc, threshold]
    return tuple(x for k in RF_CLASSES for x in best[k])


CMU_CLASSES = (('happ', 0, 0.1), ('sadn', 1, -0.3), ('ange', 2, -0.5), ('surp', 4, -0.6),
               ('disg', 3, -0.3), ('fear', 5, -0.5))                     # cmu-mosei/run.py:478-495


def cmu_test(rows):
    """cmu-mosei/run.py:456-498 over precomputed scores.

    rows: list of (preds [M][1,7] fp32 -- one batch-1 output per model, label [1,7] int64).
    Returns {name: (acc, f1)} for the six classes the reference prints."""
    lists = {k: ([], []) for k, _, _ in CMU_CLASSES}
    for preds, label in rows:
        s = preds[0]
        for p in preds[1:]:
            s = s + p
        pred = torch.mean(s / len(preds), 0)                                # :476
        label = label[0]
        for k, c, thr in CMU_CLASSES:
            hard = torch.where(pred > thr, torch.ones_like(pred), torch.zeros_like(pred))
            lists[k][0].append(int(label[c]))
            lists[k][1].append(int(hard[c]))
    return {k: (accuracy_score(*lists[k]), f1_score(*lists[k], average='weighted')) for k, _, _ in CMU_CLASSES}


def sweep_counts(preds, weights, labels, thresholds, post_div=1.0, row_mask=None, per_class=False):
    """Per-(threshold, class) confusion counts {tp, fp, fn, tn} for one call of
    mep_threshold_sweep (include/mep.h), by plain numpy loops over the same fp32 arithmetic.
    preds: list of [N, C] fp32; labels [N, C] int; thresholds [n_thr] or [n_thr, C] fp32;
    row_mask [N/P, P] int (rows count while the mask prefix is all 1)."""
    f32 = np.float32
    s = preds[0].astype(f32) * f32(weights[0])
    for p, w in zip(preds[1:], weights[1:]):
        s = (s + p.astype(f32) * f32(w)).astype(f32)
    s = (s / f32(post_div)).astype(f32)
    n, c = s.shape
    counts_row = np.ones(n, bool)
    if row_mask is not None:
        assert n == row_mask.size, (n, row_mask.shape)
        counts_row = np.cumprod(row_mask == 1, axis=1).astype(bool).reshape(-1)
    thr = np.asarray(thresholds, f32)
    n_thr = thr.shape[0]
    out = np.zeros((n_thr, c, 4), np.int64)
    pos_l = (labels != 0)[counts_row]
    sv = s[counts_row]
    for t in range(n_thr):
        tt = thr[t] if per_class else np.full(c, thr[t], f32)
        pred = sv > tt[None, :]
        out[t, :, 0] = (pos_l & pred).sum(0)
        out[t, :, 1] = (~pos_l & pred).sum(0)
        out[t, :, 2] = (pos_l & ~pred).sum(0)
        out[t, :, 3] = (~pos_l & ~pred).sum(0)
    return out, s
