"""Batch assembly: the oracle against the reference's own data-loader
output (tests/golden/batch_golden.npz, make_batch_golden.py) on the CPU; mep_assemble_windows
(mep_amd.batching) against the golden batches and the oracle on the GPU.  Bit-exact: the slots
are gathers, the summary rows max / min / frame-order mean in the source dtype."""
import numpy as np
import pytest
import torch

from oracle import batching as ob
from tests.golden import fixtures

MODS = ('linguistic', 'visual', 'acoustic')


def _golden():
    meta, g = fixtures.load('batch_golden')
    data = {m: {} for m in MODS}
    labels = {}
    for k, v in g.items():
        if k.startswith('seq/'):
            _, m, n = k.split('/')
            data[m][n] = v
        elif k.startswith('label/'):
            labels[k[6:]] = v
    cmu_labels = {k[10:]: v for k, v in g.items() if k.startswith('cmu_label/')}
    return meta, g, data, labels, cmu_labels


def _cmu_chunks(meta):
    pairs = [tuple(p) for p in meta['cmu_pairs']]
    bs = meta['cmu_batch_size']
    return [pairs[i:i + bs] for i in range(0, len(pairs), bs)]


def _lens(meta, key):
    l = meta[key]
    return l['L_LEN'], l['V_LEN'], l['A_LEN']


def _eq(got, want, name):
    got = got.cpu().numpy() if torch.is_tensor(got) else got
    assert got.shape == want.shape, (name, got.shape, want.shape)
    assert got.dtype == want.dtype, (name, got.dtype, want.dtype)
    np.testing.assert_array_equal(got, want, err_msg=name)


def test_oracle_cmu_matches_reference_loader():
    meta, g, data, _, cmu_labels = _golden()
    chunks = _cmu_chunks(meta)
    assert len(chunks) == meta['cmu_batches']
    for b, pairs in enumerate(chunks):
        out = ob.cmu_batch(data, cmu_labels, pairs, _lens(meta, 'cmu_lens'))
        for i, x in enumerate(out):
            _eq(x, g['cmu/%d/%d' % (b, i)], 'cmu batch %d col %d' % (b, i))


def test_oracle_rf_matches_reference_loader():
    meta, g, data, labels, _ = _golden()
    lists = meta['rf_lists']
    dims = tuple(meta['rf_lens'][k] for k in ('L_DIM', 'V_DIM', 'A_DIM'))
    for b in range(meta['rf_batches']):
        out = ob.rf_batch(data, {k: v[None, :][0] for k, v in labels.items()}, lists[3 * b:3 * b + 3],
                          _lens(meta, 'rf_lens'), dims)
        for i, x in enumerate(out):
            _eq(x, g['rf/%d/%d' % (b, i)], 'rf batch %d col %d' % (b, i))


# ------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_cmu_batch_gpu_matches_reference(cuda):
    from mep_amd import batching
    meta, g, data, _, cmu_labels = _golden()
    store = batching.FeatureStore(data, cuda)
    for b, pairs in enumerate(_cmu_chunks(meta)):
        out = batching.cmu_batch(store, pairs, cmu_labels, _lens(meta, 'cmu_lens'))
        torch.cuda.synchronize()
        for i, x in enumerate(out):
            _eq(x, g['cmu/%d/%d' % (b, i)], 'cmu batch %d col %d' % (b, i))


@pytest.mark.gpu
def test_rf_batch_gpu_matches_reference(cuda):
    from mep_amd import batching
    meta, g, data, labels, _ = _golden()
    store = batching.FeatureStore(data, cuda)
    lists = meta['rf_lists']
    for b in range(meta['rf_batches']):
        out = batching.rf_batch(store, lists[3 * b:3 * b + 3], labels, _lens(meta, 'rf_lens'))
        torch.cuda.synchronize()
        for i, x in enumerate(out):
            _eq(x, g['rf/%d/%d' % (b, i)], 'rf batch %d col %d' % (b, i))


@pytest.mark.gpu
@pytest.mark.parametrize('dt', [np.float32, np.float64])
def test_cmu_batch_gpu_long_sequences(cuda, dt):
    """Sequences longer than one LDS chunk (multi-chunk frame-order mean), d = 768 (3 columns per
    lane), NaN in a non-audio modality (propagates through max / min / mean), B = 64 pairs."""
    from mep_amd import batching
    rng = np.random.default_rng(9)
    dims = {'linguistic': 768, 'visual': 35, 'acoustic': 74}
    data = {m: {} for m in MODS}
    for i in range(40):
        for m, d in dims.items():
            n = int(rng.integers(1, 400))
            x = (rng.standard_normal((n, d)) * 3 + 1).astype(dt)
            if m == 'acoustic':
                x[rng.random(x.shape) < 0.01] = np.inf
                x[rng.random(x.shape) < 0.01] = np.nan
            if m == 'visual' and i == 3:
                x[n // 2, 7] = np.nan
            data[m]['s%d' % i] = x
    names = list(data['linguistic'])
    pairs = [(batching.NO_NAME if i % 7 == 0 else names[(i * 5) % 40], names[(i * 3 + 1) % 40]) for i in range(64)]
    pairs[5] = (names[3], names[3])
    labels = {n: rng.integers(0, 2, 7) for n in names}
    lens = (50, 50, 50)
    store = batching.FeatureStore(data, cuda)
    out = batching.cmu_batch(store, pairs, labels, lens)
    torch.cuda.synchronize()
    want = ob.cmu_batch(data, labels, pairs, lens)
    for i, (x, w) in enumerate(zip(out, want)):
        _eq(x, w, 'col %d' % i)


def _train_data(rng, n=40):
    dims = {'linguistic': 300, 'visual': 35, 'acoustic': 74}
    data = {m: {} for m in MODS}
    for i in range(n):
        for m, d in dims.items():
            x = rng.standard_normal((int(rng.integers(1, 120)), d)).astype(np.float32)
            if m == 'acoustic':
                x[rng.random(x.shape) < 0.01] = -np.inf
            data[m]['s%d' % i] = x
    names = list(data['linguistic'])
    pairs = [('no_name' if i % 5 == 0 else names[i - 1], names[i]) for i in range(n)]
    labels = {k: rng.integers(0, 2, 7) for k in names}
    return data, labels, pairs


@pytest.mark.gpu
def test_device_loader_trains_like_host_loader(cuda):
    """cmu train() fed by batching.cmu_data_loader (device assembly, side-stream prefetch) equals
    train() fed the reference-layout host batches (lists of per-row numpy tuples) bit for bit."""
    import random
    from mep_amd import batching, cmu_mosei
    from mep_amd.optim import FusedAdamW
    from tests.gpu_util import cmu_model
    meta, _ = fixtures.load('cmu_cfg1')
    data, labels, pairs = _train_data(np.random.default_rng(4))
    lens = (50, 50, 50)
    store = batching.FeatureStore(data, cuda)

    m1 = cmu_model(meta, cuda)
    o1 = FusedAdamW(m1, lr=1e-3)
    random.seed(3)
    loss_dev = cmu_mosei.train(m1, batching.cmu_data_loader(store, lens)(list(pairs), labels, 16), o1)

    m2 = cmu_model(meta, cuda)
    o2 = FusedAdamW(m2, lr=1e-3)
    random.seed(3)
    order = list(pairs)
    random.shuffle(order)
    host = [list(zip(*ob.cmu_batch(data, labels, order[i:i + 16], lens))) for i in range(0, len(order), 16)]
    loss_host = cmu_mosei.train(m2, host, o2)
    torch.cuda.synchronize()
    assert loss_dev == loss_host
    for (k, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k


@pytest.mark.gpu
def test_rf_device_loader_trains_like_host_loader(cuda):
    """realformer train() fed by batching.rf_data_loader equals train() fed the reference-layout
    host batches bit for bit (State_Transfer, fused Adam engine)."""
    import random
    from mep_amd import batching
    from mep_amd import realformer as rf
    from mep_amd.optim import FusedAdam
    from tests.test_gpu_realformer import _state
    meta, _ = fixtures.load('rf_state_small')
    rng = np.random.default_rng(8)
    dims = {'linguistic': 300, 'visual': 35, 'acoustic': 74}
    data = {m: {} for m in MODS}
    for i in range(12):
        for m, d in dims.items():
            x = rng.standard_normal((int(rng.integers(1, 12)), d)).astype(np.float32)
            x[rng.random(x.shape) < 0.02] = np.nan
            data[m]['u%d' % i] = x
    labels = {'u%d' % i: rng.standard_normal(7) for i in range(12)}
    lists = [['u%d' % (3 * k), 'u%d' % (3 * k + 1), 'no_name' if k == 1 else 'u%d' % (3 * k + 2)] for k in range(4)]
    lens = (6, 6, 6)
    store = batching.FeatureStore(data, cuda)

    m1 = _state(meta, cuda)
    o1 = FusedAdam(m1, lr=1e-3)
    random.seed(2)
    loss_dev = rf.train(m1, batching.rf_data_loader(store, labels, lens)(None, [list(x) for x in lists], 2), o1)

    m2 = _state(meta, cuda)
    o2 = FusedAdam(m2, lr=1e-3)
    random.seed(2)
    order = [list(x) for x in lists]
    random.shuffle(order)
    host = [list(zip(*ob.rf_batch(data, labels, order[i:i + 2], lens, tuple(dims.values()))))
            for i in range(0, len(order), 2)]
    loss_host = rf.train(m2, host, o2)
    torch.cuda.synchronize()
    assert loss_dev == loss_host
    for (k, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
