"""Batch assembly oracle (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).  SURVEY.md 8(f) row 1.

A numpy restatement of the reference's per-utterance windowing and batch composition, over a
plain dict data set (``{modality: {name: [L, d] array}}``, labels separately) instead of an mmsdk
object, and with the name order given (the reference shuffles in place first):
  * cmu_masking / cmu_batch:  cmu-mosei/run.py:104-151 (masking, is_bert=False) and :154-198
    (data_loader: previous + current utterance per row, an extra row of last windows when the
    current text has two windows, zero 'no_name' slots);
  * rf_masking / rf_batch:    others/realformer.py:72-82 (masking) and :94-125 (data_loader).
Pinned by tests/golden/batch_golden.npz, produced by the reference's own masking() / data_loader()
(AST-extracted, fed a stand-in data-set object of the same synthetic sequences;
tests/golden/make_batch_golden.py).
"""
import numpy as np

AUDIO_FILL = -71.0


def _clean(m):
    m = np.array(m, copy=True)
    bad = ~np.isfinite(m)
    m[bad] = AUDIO_FILL
    return m


def cmu_masking(m, m_len, is_audio=False):
    """cmu-mosei/run.py:104-151 (is_bert=False) -> (list of windows [m_len, d], list of masks)."""
    if is_audio:
        m = _clean(m)
    stats = np.stack([m.max(axis=0), m.min(axis=0), m.mean(axis=0)])
    if len(m) >= m_len - 3:
        first = np.concatenate([stats, m[:m_len - 3]], axis=0)
        last = np.concatenate([stats, m[len(m) - m_len + 3:]], axis=0)
        return [first, last], [np.ones(m_len), np.ones(m_len)]
    mask = np.concatenate([np.ones(len(m) + 3), np.zeros(m_len - len(m) - 3)])
    w = np.concatenate([stats, m, np.zeros((m_len - len(m) - 3, m.shape[1]))], axis=0)
    return [w], [mask]


def cmu_batch(data, labels, pairs, lens):
    """data_loader body (cmu-mosei/run.py:157-197) for one batch of (prev name or 'no_name', cur
    name) pairs; lens = (L_LEN, V_LEN, A_LEN).  Returns the 7 stacked fp32 / int64 arrays
    (l, v, a, l_mask, v_mask, a_mask, label) torch.cuda.FloatTensor would build (run.py:362)."""
    mods = ('linguistic', 'visual', 'acoustic')
    rows = []
    for prev, cur in pairs:
        w0, w1 = {}, {}
        for mod, n in zip(mods, lens):
            if prev == 'no_name':
                d = data[mod][cur].shape[1]
                w0[mod] = ([np.zeros((n, d))], [np.zeros(n)])
            else:
                w0[mod] = cmu_masking(data[mod][prev], n, is_audio=mod == 'acoustic')
            w1[mod] = cmu_masking(data[mod][cur], n, is_audio=mod == 'acoustic')
        pick = [-1, 0] if len(w1['linguistic'][1]) > 1 else [0]
        for k in pick:
            feats = [np.stack([w0[m][0][k], w1[m][0][k]]) for m in mods]
            masks = [np.stack([w0[m][1][k], w1[m][1][k]]) for m in mods]
            rows.append(feats + masks + [np.asarray(labels[cur])])
    cols = list(zip(*rows))
    return [np.stack(c).astype(np.int64 if i == 6 else np.float32) for i, c in enumerate(cols)]


def rf_masking(m, m_len):
    """others/realformer.py:72-82 on features[-m_len:] -> (window [m_len, d], mask [m_len])."""
    m = m[-m_len:]
    mask = np.ones(m_len) if len(m) >= m_len else np.concatenate([np.ones(len(m)), np.zeros(m_len - len(m))])
    w = np.concatenate([m, np.zeros((m_len, m.shape[1]))], axis=0)[:m_len]
    return _clean(w), mask


def rf_label(l):
    """label_processing (realformer.py:84-92): drop entry 0, binarise the next six (> 0)."""
    lab = np.array(l[1:], copy=True)
    lab[:6] = (lab[:6] > 0).astype(lab.dtype)
    return lab


def rf_batch(data, labels, name_lists, lens, dims):
    """data_loader body (realformer.py:97-124) -> (l, v, a, label, l_mask, v_mask, a_mask, mask)
    stacked the way torch.cuda.FloatTensor / LongTensor build them (realformer.py:307-309)."""
    mods = ('linguistic', 'visual', 'acoustic')
    rows = []
    for names in name_lists:
        f = {m: [] for m in mods}
        mk = {m: [] for m in mods}
        lab, um = [], []
        for name in names:
            if name != 'no_name':
                for m, n in zip(mods, lens):
                    w, k = rf_masking(data[m][name], n)
                    f[m].append(w)
                    mk[m].append(k)
                lab.append(rf_label(labels[name]))
                um.append(1)
            else:
                for m, n, d in zip(mods, lens, dims):
                    f[m].append(np.zeros((n, d)))
                    mk[m].append(np.zeros(n))
                lab.append(np.zeros(6))
                um.append(0)
        rows.append([np.stack(f[m]) for m in mods] + [np.stack(lab)] + [np.stack(mk[m]) for m in mods]
                    + [np.asarray(um)])
    cols = list(zip(*rows))
    return [np.stack(c).astype(np.int64 if i in (3, 7) else np.float32) for i, c in enumerate(cols)]
