"""Seeded synthetic inputs and parameters shared by the golden generator and the tests.

Only *outputs* of the reference are committed as fixtures; inputs and parameter values are
regenerated from the seeds below (numpy PCG64, platform independent), so the fixtures stay
small.  Parameter values are drawn per state_dict key (seed = base ^ crc32(key)), so they do
not depend on the order in which a model registers its parameters.
"""
import zlib

import numpy as np


def param_values(shapes, seed, overrides=None):
    """shapes: {state_dict key: shape}.  Returns {key: float32 ndarray} with values spread wide
    enough that every parameter influences the output (LayerNorm affine != identity, residual
    scalars c/a/b != 0, bilinear ``trans`` U[0,1) like torch.rand).  overrides: {key: value}
    sets whole tensors to a constant (the F7 fixtures' residual coefficients c <= -1)."""
    out = {}
    overrides = overrides or {}
    assert set(overrides) <= set(shapes), sorted(set(overrides) - set(shapes))
    for key, shape in shapes.items():
        rng = np.random.default_rng((seed * 1000003) ^ zlib.crc32(key.encode()))
        shape = tuple(shape)
        leaf = key.rsplit('.', 1)[-1]
        if key == 'trans':
            v = rng.random(shape)
        elif leaf in ('c', 'a', 'b') and len(shape) == 1 and shape[0] == 1:
            v = rng.uniform(-0.6, 0.6, shape)
        elif 'norm' in key and leaf == 'weight':
            v = 1.0 + 0.2 * rng.standard_normal(shape)
        elif leaf == 'bias':
            v = 0.2 * rng.standard_normal(shape)
        elif 'position_embeddings' in key:
            v = 0.5 * rng.standard_normal(shape)
        else:
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else shape[0]
            v = rng.standard_normal(shape) / np.sqrt(fan_in)
        if key in overrides:
            v = np.full(shape, overrides[key])
        out[key] = v.astype(np.float32)
    return out


def masks_for(rng, lead, t, min_len=1):
    """Right-padded 0/1 masks with valid length ~ U{min_len..t} per leading index."""
    lens = rng.integers(min_len, t + 1, size=lead)
    return (np.arange(t)[None, :] < lens.reshape(-1, 1)).astype(np.float32).reshape(*lead, t)


def features(rng, shape, mask=None):
    x = rng.standard_normal(shape).astype(np.float32)
    if mask is not None:           # padded frames are zero, as the reference loaders pad them
        x *= mask[..., None]
    return x


def cmu_batch(seed, B, T, dims=(300, 35, 74), no_name_rows=(0,), full_masks=False):
    """Concat_Trans batch: l/v/a [B,2,T_m,d_m], masks [B,2,T_m], int64 labels [B,7].
    Rows listed in ``no_name_rows`` get an all-zero, fully-masked previous utterance, as
    data_loader builds for the first utterance of a video (cmu-mosei/run.py:162-168)."""
    rng = np.random.default_rng(seed)
    Tl, Tv, Ta = (T, T, T) if np.isscalar(T) else T
    out = []
    for t, d in zip((Tl, Tv, Ta), dims):
        m = np.ones((B, 2, t), np.float32) if full_masks else masks_for(rng, (B, 2), t)
        x = features(rng, (B, 2, t, d), m)
        for r in no_name_rows:
            if r < B:
                m[r, 0] = 0.0
                x[r, 0] = 0.0
        out.append((x, m))
    labels = (rng.random((B, 7)) < 0.3).astype(np.int64)
    (l, lm), (v, vm), (a, am) = out
    return l, v, a, lm, vm, am, labels


def ren_batch(seed, pairs, T, dims=(768, 640, 205), n_cls=9):
    """Ren-MME batch as its data_loader emits it: every sample twice (Ren-MME/run.py:143-146).
    Returns the 12-tuple of inputs (reference argument order) and float labels [2*pairs, 9]."""
    rng = np.random.default_rng(seed)
    Tl, Tv, Ta = (T, T, T) if np.isscalar(T) else T
    parts = {}
    for side in ('pre', 'pro'):
        for name, t, d in (('text', Tl, dims[0]), ('video', Tv, dims[1]), ('audio', Ta, dims[2])):
            m = masks_for(rng, (pairs,), t)
            parts[(side, name)] = (np.repeat(features(rng, (pairs, t, d), m), 2, 0), np.repeat(m, 2, 0))
    labels = np.repeat((rng.random((pairs, n_cls)) < 0.3).astype(np.float32), 2, 0)
    order = (('pre', 'text'), ('pro', 'text'), ('pre', 'video'), ('pro', 'video'), ('pre', 'audio'), ('pro', 'audio'))
    inputs = []
    for k in order:
        inputs.extend(parts[k])
    return tuple(inputs), labels


def realformer_batch(seed, B, P, T, dims=(300, 35, 74)):
    """State_Transfer batch: l/v/a [B,P,T,d], labels int64 [B,P,6], masks [B,P,T], utterance
    mask int64 [B,P] with trailing 'no_name' utterances zeroed (others/realformer.py:102-123)."""
    rng = np.random.default_rng(seed)
    n_utt = rng.integers(1, P + 1, size=B)
    um = (np.arange(P)[None, :] < n_utt[:, None]).astype(np.int64)
    feats = []
    for d in dims:
        m = masks_for(rng, (B, P), T) * um[..., None]
        feats.append((features(rng, (B, P, T, d), m), m.astype(np.float32)))
    labels = (rng.random((B, P, 6)) < 0.3).astype(np.int64) * um[..., None]
    (l, lm), (v, vm), (a, am) = feats
    return l, v, a, labels, lm, vm, am, um


def block_inputs(seed, B, Tq, Tk, D, H, with_prev=True, mask_kind='key'):
    """Standalone Attention_Block inputs: q [B,Tq,D], kv [B,Tk,D], the mask, S_prev [B,H,Tq,Tk]
    built like a previous layer's post-mask scores, and an upstream gradient.  mask_kind: 'key'
    ([B, Tk] right-padded), 'none' (mask=None: S_prev unmasked) or 'q3' (a [B, Tq, Tk] mask,
    Bernoulli(0.7) per (query, key): the 3-D form multi_head_attention accepts, run.py:250-252)."""
    rng = np.random.default_rng(seed)
    q = rng.standard_normal((B, Tq, D)).astype(np.float32)
    kv = rng.standard_normal((B, Tk, D)).astype(np.float32)
    mask = masks_for(rng, (B,), Tk)
    if mask_kind == 'q3':
        mask = (rng.random((B, Tq, Tk)) < 0.7).astype(np.float32)
    s_prev = None
    if with_prev:
        s_prev = (0.5 * rng.standard_normal((B, H, Tq, Tk))).astype(np.float32)
        m4 = {'key': lambda: mask[:, None, None, :], 'q3': lambda: mask[:, None, :, :],
              'none': lambda: np.ones((1, 1, 1, 1), np.float32)}[mask_kind]()
        s_prev = (s_prev - np.float32(1e8) * (np.float32(1.0) - m4)).astype(np.float32)
    g_out = rng.standard_normal((B, Tq, D)).astype(np.float32)
    return q, kv, None if mask_kind == 'none' else mask, s_prev, g_out


def robot_batch(seed, B, T, dims=(768, 256, 512, 1024, 40)):
    """robot_demo.py Multi_class inputs in its forward order (robot_demo.py:390): l [B,T_l,768],
    v_256 / v_512 / v_1024 [B,T_v,d], a [B,T_a,40], then the l / v / a masks [B,T_m]."""
    rng = np.random.default_rng(seed)
    Tl, Tv, Ta = T
    lm, vm, am = masks_for(rng, (B,), Tl), masks_for(rng, (B,), Tv), masks_for(rng, (B,), Ta)
    l = features(rng, (B, Tl, dims[0]), lm)
    v256, v512, v1024 = (features(rng, (B, Tv, d), vm) for d in dims[1:4])
    a = features(rng, (B, Ta, dims[4]), am)
    return l, v256, v512, v1024, a, lm, vm, am
