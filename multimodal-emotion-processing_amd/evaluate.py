"""Evaluation: ensemble combine + threshold sweep on the GPU.

The reference evaluates by re-running the whole test set through every model once per threshold
and thresholding on the host:
  * others/realformer.py:395-477 ``test(model_1, model_2)``: 400 thresholds t/200 - 1, ensemble
    ``pred_1 * 0.6 + pred_2 * 0.4``, rows walked while ``mask[i][j] == 1``, per-class weighted F1
    and accuracy from sklearn, best threshold per class by strict ``>``;
  * cmu-mosei/run.py:456-498 ``test(model_1, .., model_4)``: batch-1 mean of 4 models, fixed
    per-class thresholds, weighted F1 / accuracy per class.
Here each model runs once per batch on the HIP plan, and ``mep_threshold_sweep`` turns the scores
into exact integer confusion counts for every (threshold, class) on the device.  The F1 / accuracy
arithmetic on those counts is the host's, as sklearn's is in the reference (weighted F1 over the
two labels {0, 1}: f1_k = 2 tp_k / (2 tp_k + fp_k + fn_k), weighted by the true support of k).

Reference behaviour kept on purpose: realformer's label/prediction lists are never reset between
thresholds (realformer.py:404-409 sit outside the ``for t`` loop), so the metrics of threshold t
cover the predictions of thresholds 0..t.  ``rf_test`` reproduces that with a prefix sum of the
counts over t; ``cumulative=False`` gives the per-threshold metrics instead.
"""
import ctypes

import numpy as np
import torch

from . import _lib

RF_CLASSES = ('happ', 'sadn', 'ange', 'surp', 'disg', 'fear')
CMU_CLASSES = (('happ', 0, 0.1), ('sadn', 1, -0.3), ('ange', 2, -0.5), ('surp', 4, -0.6),
               ('disg', 3, -0.3), ('fear', 5, -0.5))        # cmu-mosei/run.py:478-495


_HIST = {}   # (device, C, n_thr) -> zeroed int32 workspace of the sorted-threshold path


def _hist_workspace(dev, C, n_thr):
    key = (str(dev), C, n_thr)
    w = _HIST.get(key)
    if w is None:
        w = _HIST[key] = torch.zeros(C, 2, n_thr + 1, dtype=torch.int32, device=dev)
    return w


def threshold_sweep(preds, labels, thresholds, weights=None, post_div=1.0, row_mask=None,
                    counts=None, scores=None, stream=None, sorted_path=None):
    """Accumulate {tp, fp, fn, tn} for every (threshold, class) into ``counts`` [n_thr, C, 4] int32.

    preds: list of [..., C] fp32 CUDA tensors (one per model, same shape; rows may be strided);
    labels: [..., C] int64 (positive iff != 0); thresholds: [n_thr] or [n_thr, C] fp32 (per-class);
    score = (sum_m preds[m] * weights[m]) / post_div (fp32, each op rounded, in model order);
    row_mask: optional [B, P] int64 utterance mask for preds of shape [B, P, C] (a row counts while
    its mask prefix is all 1, realformer.py:423-437).  Returns counts (allocated zeroed if None).
    sorted_path: None = use the histogram formulation whenever every class's thresholds are
    non-decreasing (realformer's t/200 - 1 are) and fit its LDS budget; False = direct compares."""
    if not preds or len(preds) > _lib.EVAL_MAX_MODELS:
        raise ValueError('threshold_sweep: 1..%d models' % _lib.EVAL_MAX_MODELS)
    weights = [1.0] * len(preds) if weights is None else list(weights)
    if len(weights) != len(preds):
        raise ValueError('threshold_sweep: one weight per model')
    dev = preds[0].device
    if dev.type != 'cuda':
        raise RuntimeError('threshold_sweep: the HIP sweep needs CUDA tensors (no CPU path)')
    C = preds[0].shape[-1]
    if C > _lib.EVAL_MAX_CLASSES:
        raise ValueError('threshold_sweep: at most %d classes' % _lib.EVAL_MAX_CLASSES)
    shape = preds[0].shape
    p2 = []
    for p in preds:
        if p.shape != shape or p.dtype != torch.float32 or p.device != dev:
            raise ValueError('threshold_sweep: preds must share shape, fp32 dtype and device')
        p2.append(p.reshape(-1, C) if p.stride(-1) == 1 else p.contiguous().reshape(-1, C))
    N = p2[0].shape[0]
    ld_pred = p2[0].stride(0)
    if any(p.stride(0) != ld_pred or p.stride(1) != 1 for p in p2):
        p2 = [p.contiguous() for p in p2]
        ld_pred = C
    lab = labels.to(device=dev, dtype=torch.int64).reshape(-1, C).contiguous()
    if lab.shape[0] != N:
        raise ValueError('threshold_sweep: labels rows %d != preds rows %d' % (lab.shape[0], N))
    thr = torch.as_tensor(thresholds, dtype=torch.float32).to(dev).contiguous()
    per_class = thr.dim() == 2
    if per_class and thr.shape[1] != C:
        raise ValueError('threshold_sweep: per-class thresholds must be [n_thr, %d]' % C)
    n_thr = thr.shape[0]
    P = 0
    if row_mask is not None:
        row_mask = row_mask.to(device=dev, dtype=torch.int64).contiguous()
        P = row_mask.shape[-1]
        if row_mask.numel() != N:
            raise ValueError('threshold_sweep: row_mask has %d entries for %d rows' % (row_mask.numel(), N))
    if counts is None:
        counts = torch.zeros(n_thr, C, 4, dtype=torch.int32, device=dev)
    elif counts.shape != (n_thr, C, 4) or counts.dtype != torch.int32 or not counts.is_contiguous():
        raise ValueError('threshold_sweep: counts must be a contiguous int32 [%d, %d, 4]' % (n_thr, C))
    if scores is not None and (scores.shape[-1] != C or scores.numel() != N * C or not scores.is_contiguous()
                               or scores.dtype != torch.float32):
        raise ValueError('threshold_sweep: scores must be a contiguous fp32 tensor of %d x %d' % (N, C))
    d = _lib.SweepDesc()
    for m, p in enumerate(p2):
        d.preds[m] = p.data_ptr()
        d.weights[m] = float(weights[m])
    d.labels = lab.data_ptr()
    d.row_mask = row_mask.data_ptr() if row_mask is not None else 0
    d.thresholds = thr.data_ptr()
    d.scores = scores.data_ptr() if scores is not None else 0
    d.counts = counts.data_ptr()
    d.n_models, d.N, d.C, d.n_thr, d.P = len(p2), N, C, n_thr, P
    d.ld_pred, d.ld_label, d.post_div, d.thr_per_class = ld_pred, C, float(post_div), int(per_class)
    fits = C * (3 * n_thr + 2) * 4 <= 65536
    if sorted_path is None:
        sorted_path = fits and n_thr > 1 and bool((thr[1:] >= thr[:-1]).all())
    elif sorted_path and not (fits and bool((thr[1:] >= thr[:-1]).all())):
        raise ValueError('threshold_sweep: sorted_path needs non-decreasing thresholds within the LDS budget')
    if sorted_path:
        d.sorted, d.hist = 1, _hist_workspace(dev, C, n_thr).data_ptr()
    _lib.call('mep_threshold_sweep', ctypes.byref(d), stream=stream)
    return counts


def metrics_from_counts(counts):
    """counts [..., 4] (tp, fp, fn, tn) -> (weighted F1, accuracy) float64 arrays [...], the values
    sklearn's f1_score(average='weighted') / accuracy_score give on the same 0/1 lists."""
    c = np.asarray(counts.cpu() if torch.is_tensor(counts) else counts, dtype=np.int64)
    tp, fp, fn, tn = (c[..., i].astype(np.float64) for i in range(4))
    n = tp + fp + fn + tn
    with np.errstate(divide='ignore', invalid='ignore'):
        d1, d0 = 2 * tp + fp + fn, 2 * tn + fn + fp
        f1_pos = np.where(d1 > 0, 2 * tp / np.where(d1 > 0, d1, 1), 0.0)
        f1_neg = np.where(d0 > 0, 2 * tn / np.where(d0 > 0, d0, 1), 0.0)
        w_pos, w_neg = tp + fn, tn + fp
        f1 = np.where(n > 0, (f1_neg * w_neg + f1_pos * w_pos) / np.where(n > 0, n, 1), 0.0)
        acc = np.where(n > 0, (tp + tn) / np.where(n > 0, n, 1), 0.0)
    return f1, acc


def rf_thresholds(n_thr=400):
    return np.array([t / 200 - 1.0 for t in range(n_thr)], dtype=np.float32)


def rf_counts(model_1, model_2, iterator, n_thr=400, device='cuda'):
    """Counts [n_thr, 6, 4] (per threshold, not cumulative) of realformer's test() over one pass of
    ``iterator`` (batches as its data_loader yields them)."""
    from .realformer import _to_device
    model_1.eval()
    model_2.eval()
    thr = torch.from_numpy(rf_thresholds(n_thr)).to(device)
    counts = None
    with torch.no_grad():
        for batch in iterator:
            l, v, a, label, lm, vm, am, mask = _to_device(batch, device)
            p1 = model_1(l, v, a, lm, vm, am)
            p2 = model_2(l, v, a, lm, vm, am)
            counts = threshold_sweep([p1, p2], label, thr, weights=(0.6, 0.4), row_mask=mask, counts=counts)
    if counts is None:
        counts = torch.zeros(n_thr, len(RF_CLASSES), 4, dtype=torch.int32, device=device)
    return counts


def rf_select(counts, n_thr=400, cumulative=True):
    """counts [n_thr, 6, 4] -> realformer test()'s 18-tuple (best f1, its acc, its threshold for
    happ, sadn, ange, surp, disg, fear; realformer.py:438-477, strict > from 0)."""
    c = np.asarray(counts.cpu(), dtype=np.int64) if torch.is_tensor(counts) else np.asarray(counts, np.int64)
    if cumulative:
        c = np.cumsum(c, axis=0)
    f1, acc = metrics_from_counts(c)
    out = []
    for k in range(len(RF_CLASSES)):
        best = [0, 0, 0]
        for t in range(n_thr):
            if f1[t, k] > best[0]:
                best = [float(f1[t, k]), float(acc[t, k]), t / 200 - 1.0]
        out += best
    return tuple(out)


def rf_test(model_1, model_2, iterator, n_thr=400, cumulative=True, device='cuda'):
    """others/realformer.py:395-477: ensemble threshold sweep of two State_Transfer models."""
    return rf_select(rf_counts(model_1, model_2, iterator, n_thr, device), n_thr, cumulative)


def cmu_counts(models, iterator, device='cuda'):
    """Counts [1, 7, 4] of cmu-mosei's test() (run.py:456-498): mean of the models' logits, fixed
    per-class thresholds (class 6 is not reported; its threshold is 0)."""
    from .cmu_mosei import _to_device
    for m in models:
        m.eval()
    thr = np.zeros((1, 7), np.float32)
    for _, c, t in CMU_CLASSES:
        thr[0, c] = t
    thr = torch.from_numpy(thr).to(device)
    counts = torch.zeros(1, 7, 4, dtype=torch.int32, device=device)
    with torch.no_grad():
        for batch in iterator:
            l, v, a, lm, vm, am, label = _to_device(batch, device)
            preds = [m(l, v, a, lm, vm, am) for m in models]
            threshold_sweep(preds, label, thr, weights=[1.0] * len(preds), post_div=len(preds),
                            counts=counts)
    return counts


def cmu_test(models, iterator, device='cuda', verbose=True):
    """cmu-mosei/run.py:456-498 -> {name: (acc, f1)}; prints the reference's lines when verbose."""
    f1, acc = metrics_from_counts(cmu_counts(models, iterator, device))
    res = {k: (float(acc[0, c]), float(f1[0, c])) for k, c, _ in CMU_CLASSES}
    if verbose:
        for k in ('happ', 'sadn', 'ange', 'fear', 'disg', 'surp'):
            print('%s_acc: ' % k, res[k][0])
            print('%s_f1: ' % k, res[k][1])
    return res
