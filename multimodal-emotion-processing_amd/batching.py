"""Device-side batch assembly.

The reference builds every batch on the host: per utterance it windows and masks each modality
with numpy (``masking``), stacks the slots into Python lists and copies them with
``torch.cuda.FloatTensor(list)`` (cmu-mosei/run.py:104-198,362; others/realformer.py:72-125,
307-309).  Here the raw sequences are packed once into one HBM-resident buffer per modality
(``FeatureStore``), and a batch is one ``mep_assemble_windows`` launch that gathers, windows,
summarises (max / min / mean rows), cleans (inf / nan -> -71) and masks every slot of every
modality on the device.  Only the per-batch slot table (sequence ids and window starts, a few
hundred int32) crosses PCIe.

Row order and windows follow the reference's data loaders exactly (tests/test_batching.py pins
them against the reference's own output, tests/golden/batch_golden.npz):
  * cmu_batch:  per (previous, current) pair, a row of last windows when the current text has two
    windows (L >= L_LEN - 3), then a row of first windows; a 'no_name' previous slot is zeros.
  * rf_batch:   per list of P_LEN names, the last m_len frames of each ('no_name' -> zeros, mask 0).
"""
import ctypes

import numpy as np
import torch

from . import _lib

MODALITIES = ('linguistic', 'visual', 'acoustic')
NO_NAME = 'no_name'


class FeatureStore:
    """Packed, device-resident sequences: per modality one [n_frames, d] buffer (fp32, or fp64
    when the source arrays are fp64 -- the statistics are computed in the source dtype, as numpy
    does) plus an (offset, length) segment table; names map to sequence ids."""

    def __init__(self, data, device='cuda'):
        """data: {modality: {name: [L, d] array}} (the mmsdk ``computational_sequences[m].data[name]
        ["features"]`` arrays)."""
        self.device = torch.device(device)
        if self.device.type != 'cuda':
            raise RuntimeError('FeatureStore: device-side batch assembly needs a CUDA device')
        self.mods = {}
        for mod, seqs in data.items():
            names = list(seqs)
            arrs = [np.asarray(seqs[n]) for n in names]
            if not arrs:
                continue
            d = arrs[0].shape[1]
            f64 = any(a.dtype == np.float64 for a in arrs)
            dt = np.float64 if f64 else np.float32
            for n, a in zip(names, arrs):
                if a.ndim != 2 or a.shape[1] != d or a.shape[0] < 1:
                    raise ValueError('FeatureStore: %s/%s must be [L >= 1, %d]' % (mod, n, d))
            lens = np.array([a.shape[0] for a in arrs], np.int64)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            packed = torch.from_numpy(np.concatenate([a.astype(dt, copy=False) for a in arrs], axis=0))
            segs = torch.from_numpy(np.stack([offs, lens], axis=1).reshape(-1))
            self.mods[mod] = dict(src=packed.to(self.device), segs=segs.to(self.device), d=d, f64=f64,
                                  ids={n: i for i, n in enumerate(names)}, lens=lens)

    def length(self, mod, name):
        m = self.mods[mod]
        return int(m['lens'][m['ids'][name]])

    def dim(self, mod):
        return self.mods[mod]['d']

    def ids(self, mod, names):
        """Sequence ids of ``names`` (NO_NAME -> -1) as int32."""
        ids = self.mods[mod]['ids']
        return np.fromiter((-1 if n == NO_NAME else ids[n] for n in names), np.int32, len(names))

    def assemble(self, slots, stream=None):
        """slots: list of (modality, names, starts, m_len, summary, clean) with names a list of
        sequence names (NO_NAME for empty slots) or an int32 array of sequence ids (-1 = empty)
        -> list of (feat [n, m_len, d], mask [n, m_len]).  Every slot table of the launch goes to
        the device in one pinned copy."""
        if len(slots) > _lib.WINDOW_MAX_DESC:
            raise ValueError('assemble: at most %d slot groups per launch' % _lib.WINDOW_MAX_DESC)
        descs = (_lib.WindowDesc * len(slots))()
        tabs, outs = [], []
        for mod, names, starts, m_len, summary, clean in slots:
            sel = names if isinstance(names, np.ndarray) else self.ids(mod, names)
            st = np.asarray(starts, np.int32)
            if st.shape != sel.shape:
                raise ValueError('assemble: one window start per slot')
            tabs += [sel.astype(np.int32, copy=False), st]
        tab = torch.from_numpy(np.concatenate(tabs)).pin_memory().to(self.device, non_blocking=True)
        off = 0
        for k, (mod, names, starts, m_len, summary, clean) in enumerate(slots):
            m = self.mods[mod]
            n = len(names)
            feat = torch.empty(n, m_len, m['d'], dtype=torch.float32, device=self.device)
            mask = torch.empty(n, m_len, dtype=torch.float32, device=self.device)
            D = descs[k]
            D.src, D.segs = m['src'].data_ptr(), m['segs'].data_ptr()
            D.sel, D.start = tab.data_ptr() + 4 * off, tab.data_ptr() + 4 * (off + n)
            off += 2 * n
            D.out, D.mask = feat.data_ptr(), mask.data_ptr()
            D.n_out, D.m_len, D.d, D.src_f64 = n, m_len, m['d'], int(m['f64'])
            D.summary, D.clean, D.n_seq = int(summary), int(clean), len(m['ids'])
            outs.append((feat, mask))
        _lib.call('mep_assemble_windows', descs, len(slots), stream=stream)
        self._keep = tab        # the slot tables live until the next launch on this store
        return outs


def cmu_batch(store, pairs, label_dict, lens, device=None):
    """data_loader of cmu-mosei/run.py:154-198 for one batch of (previous, current) name pairs ->
    (l, v, a, l_mask, v_mask, a_mask, label) device tensors: l [R, 2, L_LEN, d_l], masks [R, 2, *],
    label [R, 7] int64, with R >= len(pairs) rows in the reference's order: per pair a row of last
    windows when the current text has two windows, then a row of first windows.  The slot tables
    are built with numpy (the host work per batch is a few dict lookups per pair)."""
    prevs = [p for p, _ in pairs]
    curs = [c for _, c in pairs]
    ids = {m: (store.ids(m, prevs), store.ids(m, curs)) for m in MODALITIES}
    two = _two_windows(store, ids['linguistic'][1], lens)
    reps = 1 + two.astype(np.int64)
    pair_of_row = np.repeat(np.arange(len(pairs)), reps)
    first_row = np.repeat(np.cumsum(reps) - reps, reps)
    last = (np.arange(len(pair_of_row)) == first_row) & two[pair_of_row]   # rows of last windows
    R = len(pair_of_row)
    slots = []
    for m, n in zip(MODALITIES, lens):
        sel = np.stack([ids[m][0][pair_of_row], ids[m][1][pair_of_row]], axis=1)      # [R, 2]
        L = np.where(sel >= 0, store.mods[m]['lens'][np.maximum(sel, 0)], 0)
        start = np.where(last[:, None] & (L >= n - 3), L - (n - 3), 0)
        slots.append((m, sel.reshape(-1).astype(np.int32), start.reshape(-1).astype(np.int32), n, True,
                      m == 'acoustic'))
    outs = store.assemble(slots)
    feats = [f.view(R, 2, n, f.shape[-1]) for (f, _), n in zip(outs, lens)]
    masks = [k.view(R, 2, n) for (_, k), n in zip(outs, lens)]
    lab_rows = np.stack([np.asarray(label_dict[c], np.int64) for c in curs])[pair_of_row]
    lab = torch.from_numpy(lab_rows).pin_memory().to(store.device, non_blocking=True)
    return feats + masks + [lab]


def rf_label(l):
    """label_processing of realformer.py:84-92 (drop entry 0, binarise the next six), as int64."""
    lab = np.array(l[1:], dtype=np.float64)
    lab[:6] = (lab[:6] > 0)
    return lab.astype(np.int64)


def rf_batch(store, name_lists, labels, lens):
    """data_loader of realformer.py:94-125 for one batch of P_LEN-name lists -> (l, v, a, label,
    l_mask, v_mask, a_mask, mask) device tensors (l [B, P, L_LEN, d_l], label [B, P, 6], mask [B, P])."""
    lens = dict(zip(MODALITIES, lens))
    P = len(name_lists[0])
    flat = [n for names in name_lists for n in names]
    starts = {m: [0 if n == NO_NAME else max(0, store.length(m, n) - lens[m]) for n in flat] for m in MODALITIES}
    outs = store.assemble([(m, flat, starts[m], lens[m], False, True) for m in MODALITIES])
    B = len(name_lists)
    feats = [f.view(B, P, lens[m], f.shape[-1]) for (f, _), m in zip(outs, MODALITIES)]
    masks = [k.view(B, P, lens[m]) for (_, k), m in zip(outs, MODALITIES)]
    lab = np.stack([np.zeros(6, np.int64) if n == NO_NAME else rf_label(labels[n]) for n in flat]).reshape(B, P, 6)
    um = np.array([0 if n == NO_NAME else 1 for n in flat], np.int64).reshape(B, P)
    dev = store.device
    lab_t = torch.from_numpy(lab).pin_memory().to(dev, non_blocking=True)
    um_t = torch.from_numpy(um).pin_memory().to(dev, non_blocking=True)
    return feats + [lab_t] + masks + [um_t]


# ------------------------------------------------------------------ drop-in data_loader
class DeviceBatch(tuple):
    """A batch already on the device, in the reference's column order; ``train`` / ``valid`` take
    it as it is (no zip / np.stack / H2D copy)."""


def _device_loader(chunks, build, store, prefetch):
    """Yield build(chunk) for each chunk as DeviceBatch (None -> an empty dp.HostShard), with
    chunk i+1 assembled on a side stream while the caller's step on chunk i runs."""
    from . import dp
    main = torch.cuda.current_stream(store.device)
    side = torch.cuda.Stream(store.device) if prefetch else main

    def launch(chunk):
        units, global_rows, row0 = chunk
        if not units:
            return None, None, global_rows, row0
        side.wait_stream(main)          # buffers recycled from the caller's stream are free
        with torch.cuda.stream(side):
            out = build(units)
            ev = torch.cuda.Event()
            ev.record(side)
        return out, ev, global_rows, row0

    nxt = launch(chunks[0]) if chunks else None
    for i in range(len(chunks)):
        out, ev, global_rows, row0 = nxt
        if i + 1 < len(chunks):
            nxt = launch(chunks[i + 1])
        if out is None:
            yield dp.HostShard([], global_rows, row0)
            continue
        main.wait_event(ev)
        if side is not main:
            for t in out:
                t.record_stream(main)
        b = DeviceBatch(out)
        b.global_rows = global_rows
        b.row0 = row0
        yield b


def _two_windows(store, cur_ids, lens):
    """Per pair: does the current text have two windows (cmu-mosei/run.py:172-183)?  A current
    name missing from the linguistic store (id -1) has no frames: one window."""
    ids = np.asarray(cur_ids)
    L = np.where(ids >= 0, store.mods['linguistic']['lens'][np.maximum(ids, 0)], 0)
    return L >= lens[0] - 3


def _cmu_rows(store, pairs, lens):
    """Batch rows of (previous, current) pairs: two when the current text has two windows."""
    if not pairs:
        return 0
    two = _two_windows(store, store.ids('linguistic', [c for _, c in pairs]), lens)
    return int(len(pairs) + two.sum())


def cmu_data_loader(store, lens, prefetch=True):
    """-> ``data_loader(name_list, label_dict, batch_size)`` with the signature and row order of
    cmu-mosei/run.py:154-198 (``random.shuffle`` of ``name_list`` in place, batches of
    ``batch_size`` (previous, current) pairs), yielding DeviceBatch.  With ``prefetch`` batch i+1 is
    assembled on a side stream while the caller's step on batch i runs on the current stream.
    Under data parallelism (mep_amd.dp) ``batch_size`` is per rank: global batch k holds pairs
    [k B W, (k+1) B W) of rank 0's shuffled order, rank r assembles pairs [r B, (r+1) B) of it and
    each DeviceBatch carries ``global_rows`` (rows of the whole global batch) for the loss scale."""
    from . import dp

    def data_loader(name_list, label_dict, batch_size):
        dp.shared_shuffle(name_list)
        w = dp.world()
        step = batch_size * w
        chunks = []
        for i in range(0, len(name_list), step):
            g = name_list[i:i + step]
            lo, hi = dp.rank_range(len(g), batch_size)
            chunks.append((g[lo:hi], _cmu_rows(store, g, lens) if w > 1 else None,
                           _cmu_rows(store, g[:lo], lens) if w > 1 else 0))
        return _device_loader(chunks, lambda pairs: cmu_batch(store, pairs, label_dict, lens), store, prefetch)

    return data_loader


def rf_data_loader(store, labels, lens, prefetch=True):
    """-> ``data_loader(data_set, name_list, batch_size)`` with the signature and row order of
    others/realformer.py:94-125 (``random.shuffle`` in place; ``data_set`` is not read -- the
    sequences live in ``store``, the label rows in ``labels[name]``), yielding DeviceBatch of
    (l, v, a, label, l_mask, v_mask, a_mask, mask); batch i+1 is assembled on a side stream
    while the caller's step on batch i runs.  Under data parallelism ``batch_size`` groups per
    rank, sharded as cmu_data_loader shards pairs."""
    from . import dp

    def data_loader(data_set, name_list, batch_size):
        dp.shared_shuffle(name_list)
        w = dp.world()
        step = batch_size * w
        chunks = []
        for i in range(0, len(name_list), step):
            g = name_list[i:i + step]
            lo, hi = dp.rank_range(len(g), batch_size)
            chunks.append((g[lo:hi], len(g) if w > 1 else None, lo))
        return _device_loader(chunks, lambda lists: rf_batch(store, lists, labels, lens), store, prefetch)

    return data_loader
