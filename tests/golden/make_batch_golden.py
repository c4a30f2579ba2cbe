"""Generate tests/golden/batch_golden.npz: the reference's own masking() / data_loader() output
for seeded synthetic sequences (runs HERE only; /root/reference does not exist on the GPU box).

The functions are AST-extracted from cmu-mosei/run.py and others/realformer.py (make_golden.
load_reference) and called on a stand-in data-set object that exposes the synthetic sequences the
way mmsdk does (``data_set.computational_sequences[mod].data[name]["features"]``).  random.shuffle
is seeded and the shuffled name order recorded, so the oracle / device path rebuild the batches in
the reference's row order.  Usage: python tests/golden/make_batch_golden.py
"""
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden.make_golden import load_reference  # noqa: E402

DIMS = {'linguistic': 300, 'visual': 35, 'acoustic': 74}
DTYPES = {'linguistic': np.float32, 'visual': np.float64, 'acoustic': np.float32}
CMU_LENS = {'L_LEN': 8, 'V_LEN': 12, 'A_LEN': 16}
RF_LENS = {'L_LEN': 8, 'V_LEN': 12, 'A_LEN': 16, 'P_LEN': 3, 'L_DIM': 300, 'V_DIM': 35, 'A_DIM': 74}
# frame counts per utterance and modality: short, exactly m_len - 3, m_len - 4, m_len, long
LENGTHS = [(3, 5, 20), (5, 9, 13), (4, 8, 12), (8, 12, 16), (30, 40, 50), (1, 1, 1), (6, 2, 14)]


class _Seq:
    def __init__(self, d):
        self.data = {k: {'features': v} for k, v in d.items()}


class _DataSet:
    def __init__(self, mods):
        self.computational_sequences = {m: _Seq(d) for m, d in mods.items()}


def sequences(seed):
    rng = np.random.default_rng(seed)
    data = {m: {} for m in DIMS}
    for i, lens in enumerate(LENGTHS):
        for (m, d), n in zip(DIMS.items(), lens):
            x = (rng.standard_normal((n, d)) * 2).astype(DTYPES[m])
            if m == 'acoustic' and n > 2:
                x[1, 3] = np.inf
                x[n - 1, 0] = -np.inf
                x[0, 5] = np.nan
            data[m]['u%d' % i] = x
    labels = {'u%d' % i: rng.standard_normal(7) for i in range(len(LENGTHS))}
    return data, labels


def main():
    out = {}
    data, labels = sequences(20261016)
    for m, d in data.items():
        for k, v in d.items():
            out['seq/%s/%s' % (m, k)] = v
    for k, v in labels.items():
        out['label/' + k] = v
    meta = {'kind': 'batch'}

    # cmu-mosei: name_list of (previous, current) pairs, label_dict[current] = 7 ints
    ns = load_reference('cmu', dict(CMU_LENS))
    ns['random'] = random
    ns['data_set'] = _DataSet(data)
    names = sorted(data['linguistic'])
    pairs = [('no_name', names[0])] + [(names[i - 1], names[i]) for i in range(1, len(names))]
    label_dict = {k: (np.abs(v[:7]) > 1).astype(np.int64) for k, v in labels.items()}
    random.seed(5)
    batches = list(ns['data_loader'](pairs, label_dict, 3))
    meta['cmu_pairs'] = [list(p) for p in pairs]          # shuffled in place by data_loader
    meta['cmu_batch_size'] = 3
    meta['cmu_lens'] = CMU_LENS
    for b, batch in enumerate(batches):
        for i, col in enumerate(zip(*batch)):
            out['cmu/%d/%d' % (b, i)] = np.stack(col).astype(np.int64 if i == 6 else np.float32)
    for k, v in label_dict.items():
        out['cmu_label/' + k] = v
    meta['cmu_batches'] = len(batches)

    # realformer: name lists of P_LEN names ('no_name' padded), labels from the label sequence
    ns = load_reference('realformer', dict(RF_LENS))
    ns['random'] = random
    mods = dict(data)
    mods['label'] = {k: v[None, :] for k, v in labels.items()}
    lists = [['u0', 'u1', 'u2'], ['u3', 'no_name', 'no_name'], ['u4', 'u5', 'u6'], ['u6', 'u1', 'no_name']]
    random.seed(6)
    batches = list(ns['data_loader'](_DataSet(mods), lists, 3))
    meta['rf_lists'] = lists
    meta['rf_lens'] = RF_LENS
    meta['rf_batches'] = len(batches)
    for b, batch in enumerate(batches):
        for i, col in enumerate(zip(*batch)):
            out['rf/%d/%d' % (b, i)] = np.stack(col).astype(np.int64 if i in (3, 7) else np.float32)
    out['meta'] = np.array(json.dumps(meta))
    path = os.path.join(HERE, 'batch_golden.npz')
    np.savez_compressed(path, **out)
    print('wrote', path, os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    main()
