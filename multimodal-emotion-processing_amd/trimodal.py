"""Execution plan of the tri-modal encoder pair + fusion head (cmu-mosei Concat_Trans,
Ren-MME Base_model) on libmep_hip.

A plan is built once per (batch, sequence lengths) shape.  It owns every activation and
gradient buffer of a training step in HBM and the device-resident descriptor arrays of each
grouped launch, so a step is a fixed sequence of ~20 launches with no host work -- capturable
as one hipGraph.

Step anatomy (reference call stack: SURVEY.md section 3A; cmu-mosei/run.py:329-369)
  forward   unify GEMM (both encoders x 3 modalities in ONE launch)  [+ shared LayerNorm, Ren]
            per layer: attention core (all 9 chains x 2 encoders in one launch),
                       block epilogue (proj -> cat -> minus -> LayerNorm, one launch)
            mean+max pool (one launch) -> fused head + circle loss (+R-Drop) + head backward
  backward  per layer (reverse): epilogue backward (from the pool's gradient), attention
            backward; per-modality gradient sum; all weight gradients in one split-K launch +
            one reduce; LayerNorm / residual-coefficient column sums.
Independent work is batched into grouped launches (grid.y = descriptor), never looped in
Python.  HBM layout: block outputs are written straight into the pooled tensor
[B, T_l+T_a+T_v, 3*n_layers*D] at their (time, feature) offsets (torch.cat at run.py:314-317 is
never materialised); inputs stay in the reference's [B, 2, T, d] (prev, cur) layout and are read
through strided row views.
"""
import ctypes
import functools

import torch

from . import _lib
from ._lib import (AttnBwdDesc, AttnDesc, ColsumDesc, DescArray, EpiBwdDesc, EpiDesc, GemmDesc,
                   HeadDesc, LnDesc, PoolDesc, Rows, SumDesc, WgradDesc, launch)

CHAINS = (('l', 'l'), ('l', 'v'), ('l', 'a'),
          ('v', 'v'), ('v', 'l'), ('v', 'a'),
          ('a', 'a'), ('a', 'l'), ('a', 'v'))          # cmu-mosei/run.py:279-313
MODS = ('l', 'v', 'a')
TIME_ORDER = ('l', 'a', 'v')                          # cmu-mosei/run.py:317
UNIFY_NAMES = {'l': 'linguistic', 'v': 'visual', 'a': 'acoustic'}


def _norm_args(plan):
    """the (norm, step, hyper) arguments of mep_reduce_grads: the optimizer workspace pointers when
    the plan's engine folds the clip's norm pass into the reduction (TrainEngine, single process)"""
    nf = plan.norm_fold
    return (None, None, None) if nf is None else tuple(ctypes.c_void_p(x) for x in nf)


def cdiv(a, b):
    return (a + b - 1) // b


WG_WAVES = 4              # csrc/gemm.hip k_wgrad: waves per workgroup (token quarters of a split)
WG_TARGET = _lib.N_CU      # workgroups per launch: one per CU (4 waves of ~400 registers)
WG_TARGET_OVERRIDE = int(_lib.switch('MEP_WG_TARGET', '0')) or None   # development: another k_wgrad workgroup count
# the pool's backward formed inside the epilogue backward (0: a separate mep_pool_bwd into dXcat)
POOL_FOLD = _lib.switch('MEP_POOL_FOLD', '1') != '0'
# mep_unify workgroups in XCD-contiguous descriptor order (xcd_order); 0: descriptor-major by id
UNIFY_XCD = _lib.switch('MEP_UNIFY_XCD', '1') != '0'


def wgrad_geometry(N, ktot, bf16=False):
    """(row tiles MT, column tiles per group KT, column groups) of k_wgrad's 32x32 tiling of an
    N x ktot weight gradient (csrc/gemm.hip wg_kt)."""
    mt = cdiv(N, 32)
    kt = _wg_kt(mt, bool(bf16))
    return mt, kt, cdiv(cdiv(ktot, 32), kt)


@functools.lru_cache(maxsize=None)
def _wg_kt(mt, bf16):
    return int(_lib.lib().mep_wgrad_kt(mt, int(bf16)))


def wg_target(bf16=False):
    """workgroups of a k_wgrad launch: one per CU times the instance's occupancy (MEP_WG_OCC; the
    bf16-path instance runs one per CU)"""
    return WG_TARGET_OVERRIDE or WG_TARGET * int(_lib.lib().mep_wgrad_occupancy(int(bool(bf16))))


def _wgrad_units(items, bf16=False):
    units = []
    for i, (_, N, n, bs, _) in enumerate(items):
        mt, kt, ncg = wgrad_geometry(N, sum(b[1] for b in bs), bf16)
        for cg in range(ncg):
            if n > 0:
                units.append((i, cg, n))
    return units


# k_wgrad cost per workgroup ~ a * tokens + c (cfg3 / cfg5 bf16 fits, round 4: a = 8.5 ns per
# token, c = 16 us of setup + partial write); in tokens, c / a:
WG_SETUP_TOKENS = int(_lib.switch('MEP_WG_SETUP_TOKENS', '1900'))


def _wgrad_fit(units, n_wg):
    """the smallest multiple of 8 tokens per segment that keeps the units within n_wg segments"""
    lo, hi = 1, cdiv(max([n for (_, _, n) in units] or [8]), 8)   # in units of 8 tokens
    while lo < hi:                        # the segment count only falls as the chunk grows
        mid = (lo + hi) // 2
        if sum(cdiv(n, 8 * mid) for (_, _, n) in units) <= n_wg:
            hi = mid
        else:
            lo = mid + 1
    return 8 * lo


def wgrad_chunk(items, n_wg=WG_TARGET, bf16=False):
    """Tokens per segment: n_wg workgroups are resident at once.  bf16 instance (one workgroup per
    CU): of the chunks that fill 1, 2, 3 or 4 such rounds, the one with the least modelled time
    rounds x (chunk + WG_SETUP_TOKENS) -- one round is the usual answer (cfg3: 1,072 tokens), but
    cfg5's 9,600-token spans would fill only 160 of 256 CUs in one round, and two rounds of 3,200
    run 98 -> 87 us.  The fp32 instance (two per CU) keeps one round: two measured slower at cfg5
    (259 vs 254 us)."""
    items = [tuple(it) + (0,) * (5 - len(it)) for it in items]
    units = _wgrad_units(items, bf16)
    if WG_TARGET_OVERRIDE or not bf16:
        return _wgrad_fit(units, n_wg)
    best = None
    for r in (1, 2, 3, 4):
        ch = _wgrad_fit(units, r * n_wg)
        cost = r * (ch + WG_SETUP_TOKENS)
        if best is None or cost < best[0]:
            best = (cost, ch)
    return best[1]


# per-(item, column group) segment counts, cost-weighted over every workgroup slot (0: one token
# chunk for the whole launch, wgrad_chunk)
WG_BALANCE = _lib.switch('MEP_WG_BALANCE', '1') != '0'


def wgrad_counts(items, n_wg=WG_TARGET, bf16=False):
    """Segments per (item, column group) unit, {(i, cg): k}: every unit's span cut into k near-equal
    chunks so that the launch fills its rounds of n_wg workgroup slots exactly and the costliest
    segment is as cheap as it can be.  A segment's cost is its tokens x (MT + KT), the 32 x 32
    operand tiles a token loads (and multiplies): a unit with fewer column tiles (the last column
    group of a 96- or 74-wide weight, one tile) gets fewer, longer segments.  One uniform chunk
    left 88 of the 512 fp32 slots empty at cfg3: the workgroups alone on a CU finished their 800
    tokens in 60% of the time of those that share one (scripts/wg_trace.py), and the shared ones
    bound the launch.  Rounds as wgrad_chunk: the bf16 instance picks 1-4 by rounds x (segment +
    WG_SETUP_TOKENS), the fp32 instance one."""
    import heapq
    items = [tuple(it) + (0,) * (5 - len(it)) for it in items]
    units = []
    for i, (_, N, n, bs, _) in enumerate(items):
        mt, kt, ncg = wgrad_geometry(N, sum(b[1] for b in bs), bf16)
        ktiles = cdiv(sum(b[1] for b in bs), 32)
        for cg in range(ncg):
            if n > 0:
                units.append(((i, cg), n, mt + min(kt, ktiles - cg * kt)))

    def fill(budget):
        k = {u: 1 for (u, _, _) in units}
        heap = [(-(n * c), u, n, c) for (u, n, c) in units]
        heapq.heapify(heap)
        total = len(units)
        while heap and total < budget:
            _, u, n, c = heapq.heappop(heap)
            if n < 8 * (k[u] + 1):            # chunks stay >= 8 tokens
                continue
            k[u] += 1
            total += 1
            heapq.heappush(heap, (-(n * c / k[u]), u, n, c))
        worst = max((cdiv(n, k[u]) * c for (u, n, c) in units), default=0)
        return worst, k
    if not units:
        return {}
    setup = WG_SETUP_TOKENS * 5   # tokens x tiles, the MT + KT = 5 tiles of a cfg3 segment
    best = None
    for r in ((1, 2, 3, 4) if bf16 and not WG_TARGET_OVERRIDE else (1,)):
        worst, k = fill(r * n_wg)
        cost = r * (worst + setup)
        if best is None or cost < best[0]:
            best = (cost, k)
    return best[1]


def wgrad_segments(items, n_wg=WG_TARGET, tok_per_split=None, bf16=False, counts=None):
    """Split every (item, column group) token span into segments of at most tok_per_split tokens,
    one segment per workgroup; counts (or, tok_per_split and counts None, wgrad_counts under
    WG_BALANCE): k segments per (item, column group); tok_per_split: chunks of at most that many
    tokens (MEP_WG_BALANCE=0: the smallest multiple of 8 that keeps the launch within n_wg
    workgroups).  A span is cut into near-equal pieces at multiples of 8.  The loop
    is bound by HBM traffic and the operand-load rate, so more, smaller segments only add setup
    and partial-reduction work (~10 us per workgroup, round-3 per-workgroup traces).
    -> (per-workgroup segment lists [(item, cg, t0, t1, slot)], slots per item)."""
    units = _wgrad_units(items, bf16)
    if tok_per_split is None and counts is None:
        if WG_BALANCE:
            counts = wgrad_counts(items, n_wg, bf16)
        else:
            tok_per_split = wgrad_chunk(items, n_wg, bf16)
    bins = []
    for (i, cg, n) in units:
        if counts is not None:
            k = counts[(i, cg)]
        else:
            tps = tok_per_split[i] if isinstance(tok_per_split, (list, tuple)) else tok_per_split
            k = cdiv(n, tps)
        # k near-equal chunks, cut at multiples of 8
        cuts = [min(n, cdiv(n * q, 8 * k) * 8) for q in range(k)] + [n]
        bins += [[(i, cg, a, b)] for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    slots = [0] * len(items)
    count = {}
    segs = []
    for b in bins:
        out = []
        for (i, cg, t0, t1) in b:
            s = count.get((i, cg), 0)
            count[(i, cg)] = s + 1
            slots[i] = max(slots[i], s + 1)
            out.append((i, cg, t0, t1, s))
        segs.append(out)
    if WG_XCD_PAIR:
        segs = _xcd_pairs(segs, n_wg)
    return segs, slots


WG_XCD_PAIR = _lib.switch('MEP_WG_XCD', '1') != '0'


def _xcd_pairs(segs, n_wg):
    """Workgroup order that puts the column groups of one token chunk on one XCD: blocks b and
    b + 8 share an XCD (round-robin dispatch, MI355X_MICROARCH.md section Workgroup dispatch), so
    member r of chunk group q (same item and tokens, column group r: the same A rows) goes to
    block 8 r + q of its 8-group block and the A operand is read from HBM once and hit in that
    XCD's L2 by the other column groups, which stream it at the same time.  Empty workgroups pad
    a short last block; the plain order is kept when the padding would exceed n_wg."""
    groups, order = {}, []
    for seg in segs:
        (i, cg, t0, t1, s), = seg
        key = (i, t0, t1)
        if key not in groups:
            groups[key] = []
            order.append(key)
        groups[key].append(seg)
    by_m = {}
    for key in order:
        by_m.setdefault(len(groups[key]), []).append(groups[key])
    out = []
    for m in sorted(by_m):
        gl = by_m[m]
        if m == 1:
            out += [g[0] for g in gl]
            continue
        for b0 in range(0, len(gl), 8):
            blk = gl[b0:b0 + 8]
            for r in range(m):
                out += [blk[q][r] if q < len(blk) else [] for q in range(8)]
    if len(out) > max(n_wg, len(segs)):
        # few, large chunk groups (cfg5: one chunk per item, 4-24 column groups each): the 8-group
        # blocks would pad past the launch, so pack whole groups onto the 8 XCDs instead
        return _xcd_pack([groups[k] for k in order], n_wg, segs)
    return out


def _xcd_pack(groups, n_wg, segs):
    """Every chunk group whole on one XCD (workgroup ids x, x + 8, x + 16, ...), groups dealt
    largest first to the XCD with the fewest workgroups so far; the XCD lists interleave into the
    launch order, short lists padded with empty workgroups.  Without it the column groups of one
    chunk land on every XCD and each streams the shared A rows from HBM (cfg5 k_wgrad: 2.9x the
    algorithmic bytes).  Falls back to the plain order if the padding would push the
    launch past n_wg."""
    lists = [[] for _ in range(8)]
    for g in sorted(groups, key=len, reverse=True):
        x = min(range(8), key=lambda i: (len(lists[i]), i))
        lists[x] += g
    depth = max(len(l) for l in lists)
    if 8 * depth > max(n_wg, len(segs)):
        return segs
    return [lists[x][j] if j < len(lists[x]) else [] for j in range(depth) for x in range(8)]


UN_LDS = 30720   # csrc/gemm.hip k_unify: floats of LDS for the staged weight


def make_unify(descs, dev, n_wg=_lib.N_CU):
    """mep_unify launch for bias-free forward projections (GemmDesc, w_nt=1, N in {32,..,128}):
    -> (descriptor array followed by the task map, workgroups).  Workgroups (one per CU: the
    staged weight holds 120 KB of LDS) are shared out over the descriptors in proportion to
    their MFMA work (16-token tiles x 16-wide k blocks)."""
    ntiles, cost = [], []
    for d in descs:
        assert d.w_nt == 1 and d.N in (16, 32, 48, 64, 96, 128) and not d.accumulate and not d.relu
        assert d.bias == 0 and d.alpha == 1.0 and d.y.ptr % 16 == 0 and d.y.sB % 4 == 0 and d.y.sT % 4 == 0
        kb = cdiv(d.K, 16)
        xv = d.K % 4 == 0 and d.x.ptr % 16 == 0 and d.x.sB % 4 == 0 and d.x.sT % 4 == 0
        if d.N * (16 * kb + 8) > UN_LDS:   # weight read from L2: 16-byte fragments, no k tail
            assert d.K % 16 == 0 and d.ldw % 4 == 0 and d.w % 16 == 0 and xv, 'mep_unify: unsupported shape'
        assert 4 * ((cdiv(d.ntok, d.x.T) - 1) * d.x.sB + (d.x.T - 1) * d.x.sT + d.K) < 2 ** 31
        ntiles.append(cdiv(d.ntok, 16))
        cost.append(ntiles[-1] * kb)
    total = float(sum(cost))
    nw = [max(1, min(cdiv(t * 2, 8), int(round(n_wg * c / total)))) for t, c in zip(ntiles, cost)]
    while sum(nw) > n_wg:
        i = max(range(len(nw)), key=lambda j: (nw[j], -cost[j]))
        nw[i] -= 1
    assert all(0 < w < 1024 for w in nw) and len(descs) < 2048
    tasks = [(i << 20) | (w << 10) | k for i, w in enumerate(nw) for k in range(w)]
    if UNIFY_XCD:
        tasks = xcd_order(tasks)
    return DescArray(GemmDesc, descs, dev, tail=tasks), len(tasks)


def xcd_order(work):
    """work list -> launch order: workgroups go to the 8 XCDs round-robin by id, so XCD x (ids x,
    x + 8, ...) receives the x-th contiguous run of the list (csrc/block.hip epi_slot): the
    workgroups of one descriptor share an XCD and its L2 for the weight they stage"""
    G = len(work)
    q, r = divmod(G, 8)
    return [work[(i % 8) * q + min(i % 8, r) + i // 8] for i in range(G)]


def make_wgrad(items, dev, tok_per_split=None, bf16=False, counts=None):
    """items: [(a_rows, N, ntok, [(b_rows, K, out_ptr, ldo), ...][, out_trans]), ...] ->
    (workspace, descs, wgrad workgroups, reduce tiles).  One descriptor per A operand; its B operands
    concatenate on K.  out_trans: dW written transposed (out[k * ldo + n]).  tok_per_split: None =
    the launch's work balanced over one workgroup per CU (wgrad_segments), else fixed token
    chunks.  bf16: plain bf16 operands (the bf16 path) instead of the 3-part split."""
    items = [tuple(it) + (0,) * (5 - len(it)) for it in items]
    segs, slots = wgrad_segments(items, n_wg=wg_target(bf16), tok_per_split=tok_per_split, bf16=bf16, counts=counts)
    total = sum(max(1, s) * N * sum(b[1] for b in bs) for s, (_, N, n, bs, _) in zip(slots, items))
    ws = torch.zeros(max(total, 1), dtype=torch.float32, device=dev)   # unwritten slots stay 0
    descs, off, rmax = [], 0, 0
    for ns, (a, N, n, bs, trans) in zip(slots, items):
        assert N <= 128 and len(bs) <= _lib.WG_MAX_B
        # k_wgrad: every 32-column tile reads one operand (wave-uniform buffer resource)
        assert all(b[1] % 32 == 0 for b in bs[:-1]), 'wgrad B operand boundaries must be multiples of 32'
        ktot = sum(b[1] for b in bs)
        for v, w in [(a, N)] + [(b[0], b[1]) for b in bs]:
            # k_wgrad: one token -> (b, t) map for every view of the item; 32-bit byte offsets
            assert v.T == a.T, 'wgrad views of one item must share T'
            assert 4 * ((cdiv(n, v.T) - 1) * v.sB + (v.T - 1) * v.sT + w) < 2 ** 31
            if bf16:   # bf16 rows read as column-pair dwords: 4-byte aligned rows, linear views
                assert v.ptr % 4 == 0 and v.sB % 2 == 0 and v.sT % 2 == 0, 'bf16 wgrad rows must be 4-byte aligned'
                assert v.T == 1 or v.sB == v.T * v.sT, 'bf16 wgrad views must be linear in the token' 
        ns = max(1, ns)
        pad = [(Rows(), 0, 0, 0)] * (_lib.WG_MAX_B - len(bs))
        allb = list(bs) + pad
        descs.append(WgradDesc(a=a, b=(Rows * _lib.WG_MAX_B)(*[b[0] for b in allb]),
                               out=(ctypes.c_uint64 * _lib.WG_MAX_B)(*[b[2] for b in allb]),
                               kb=(ctypes.c_int32 * _lib.WG_MAX_B)(*[b[1] for b in allb]),
                               ldo=(ctypes.c_int32 * _lib.WG_MAX_B)(*[b[3] for b in allb]),
                               partial=ws.data_ptr() + 4 * off, n_b=len(bs), ntok=n, N=N, Ktot=ktot,
                               tok_per_split=0, n_split=ns, accumulate=0, out_trans=int(trans),
                               # the bf16-path instance: bf16 operands from bf16 rows
                               bf16=(_lib.BF16_OPS | _lib.BF16_STORE) if bf16 else 0))
        off += ns * N * ktot
        rmax = max(rmax, cdiv(N * ktot, 256))
    assert len(descs) < 2 ** 23 and all(cg < 256 for b in segs for (_, cg, _, _, _) in b)
    offs, flat = [0], []
    for b in segs:
        for (i, cg, t0, t1, s) in b:
            flat += [(i << 8) | cg, t0, t1, s]
        offs.append(offs[-1] + len(b))
    arr = DescArray(WgradDesc, descs, dev, tail=offs + flat)
    arr.prec = _lib.PREC_BF16 if bf16 else 0   # the mep_wgrad instance (launch reads it)
    return ws, arr, len(segs), rmax


def reduce_map(wgrad, colsum, head, dev):
    """The job list of a mep_reduce_grads_mapped launch: the head-parameter blocks (head: HeadDesc
    or None), every split-sum block of each weight-gradient descriptor (1,024 entries each), every
    32-column tile of each column sum -- only real jobs, kind << 30 | descriptor << 12 | block.
    -> (device uint32 map, block count)"""
    import numpy as np
    jobs = []
    if head is not None:
        jobs += [j for j in range(_lib.lib().mep_reduce_grads_grid(0, 0, 0, 0, ctypes.byref(head)))]
    for i, d in enumerate(wgrad.items if wgrad is not None else []):
        jobs += [(1 << 30) | (i << 12) | b for b in range(cdiv(d.N * d.Ktot, 1024))]
    for i, c in enumerate(colsum.items if colsum is not None else []):
        jobs += [(2 << 30) | (i << 12) | b for b in range(cdiv(c.n_cols, 32))]
    assert all((j & 0xfff) < 4096 and ((j >> 12) & 0x3ffff) < (1 << 18) for j in jobs)
    arr = np.array(jobs or [0], dtype=np.uint32).view(np.int32)
    return torch.from_numpy(arr.copy()).to(dev), len(jobs)


# 0: the rectangular mep_reduce_grads grid (A/B runs)
REDUCE_MAP = _lib.switch('MEP_REDUCE_MAP', '1') != '0'


def reduce_rect_blocks(wgrad, colsum, head):
    """blocks of the rectangular mep_reduce_grads grid over the same descriptors"""
    wt = max((cdiv(d.N * d.Ktot, 256) for d in (wgrad.items if wgrad is not None else [])), default=0)
    ct = max((cdiv(c.n_cols, 32) for c in (colsum.items if colsum is not None else [])), default=0)
    return _lib.lib().mep_reduce_grads_grid(wgrad.n if wgrad is not None else 0, wt,
                                            colsum.n if colsum is not None else 0, ct,
                                            ctypes.byref(head) if head is not None else None)


def reduce_blocks(wgrad, colsum, head, bmap):
    """blocks (= norm partials) of the step's reduction launch"""
    return bmap[1] if REDUCE_MAP else reduce_rect_blocks(wgrad, colsum, head)


def reduce_mapped(wgrad, colsum, head, head_grads, norm, bmap, stream=None):
    """one mep_reduce_grads_mapped launch over reduce_map's jobs (bmap = (map, blocks)); with
    REDUCE_MAP off the rectangular mep_reduce_grads launch"""
    m, n = bmap
    if not REDUCE_MAP:
        wt = max((cdiv(d.N * d.Ktot, 256) for d in (wgrad.items if wgrad is not None else [])), default=0)
        ct = max((cdiv(c.n_cols, 32) for c in (colsum.items if colsum is not None else [])), default=0)
        hg = [int(x) for x in head_grads] if head is not None else [0] * 8
        _lib.call('mep_reduce_grads', wgrad.ptr if wgrad is not None else None, wgrad.n if wgrad is not None else 0, wt,
                  colsum.ptr if colsum is not None else None, colsum.n if colsum is not None else 0, ct,
                  ctypes.byref(head) if head is not None else None, *hg, *norm, stream=stream)
        return
    if n == 0:
        return
    hg = [int(x) for x in head_grads] if head is not None else [0] * 8
    _lib.call('mep_reduce_grads_mapped', wgrad.ptr if wgrad is not None else None,
              colsum.ptr if colsum is not None else None, ctypes.byref(head) if head is not None else None,
              *hg, *norm, ctypes.c_void_p(m.data_ptr()), int(n), stream=stream)


def rows(t, T, sB, sT, off=0):
    """row view of tensor t (strides and offset in elements: 4-byte fp32 or 2-byte bf16 rows);
    the kernels' 24-bit row addressing (include/mep.h mep_rows) bounds the strides and offsets"""
    if not (0 <= sB < 1 << 24 and 0 <= sT < 1 << 24 and t.numel() - off <= 1 << 32):
        raise ValueError('row view out of the kernels\' addressing range: sB %d, sT %d, %d elements'
                         % (sB, sT, t.numel() - off))
    return Rows(ptr=t.data_ptr() + t.element_size() * off, sB=sB, sT=sT, T=T)


def crows(t, T, D, off=0):
    """contiguous [B*T, D] view"""
    return rows(t, T, T * D, D, off)


class TriModalSpec:
    """Static description of one model family instance."""

    def __init__(self, D, H, n_layers, dims, NC, variant='cmu', drop_p=0.0):
        assert D == 16 * H and D % 32 == 0 and D <= 128, 'kernels need hd = 16 and D in {32,64,96,128}'
        self.D, self.H, self.nl, self.dims, self.NC = D, H, n_layers, tuple(dims), NC
        self.variant = variant                      # 'cmu' | 'ren'
        self.unify_norm = variant == 'ren'          # Ren-MME/run.py:164-166
        self.block_norm = 'norm2' if variant == 'ren' else 'norm1'
        self.head_norm = 'norm3' if variant == 'ren' else 'norm1'
        self.drop_p = float(drop_p)
        self.prefixes = ('intensity.', 'stimulation.')

    @staticmethod
    def bucket_a(name):
        """Parameters whose gradients are complete after the last epilogue backward: the blocks'
        proj / minus / LayerNorm weights and the fusion head (its gradient partials come from the
        forward's fused head kernel).  The rest -- unify weights (+ Ren-MME's unify LayerNorm) and
        the residual coefficients c (attention backward) -- is bucket B."""
        if 'multimodal_blocks.' in name:
            return not name.endswith('.c')
        return 'unify_dimension.' not in name

    def no_grad_params(self):
        """c of the first layer of every chain never receives a gradient (scores is None)."""
        out = []
        for pre in self.prefixes:
            for j in range(9):
                out.append(pre + 'multimodal_blocks.%d.c' % (self.nl * j))
        return out


class TriModalPlan:
    def __init__(self, spec, flat, B, T, device, labels_float=False, bf16=False, seed_state=None):
        """bf16: the bf16 path (include/mep.h MEP_PREC_BF16) -- unify, attention, block epilogue and
        weight-gradient products on plain bf16 operands with fp32 accumulation; storage, softmax,
        LayerNorm, pool, head, loss and AdamW in fp32.  Default: the fp32 path (1e-4 parity)."""
        self.spec, self.flat, self.B = spec, flat, B
        self.bf16 = bool(bf16)
        self.prec = _lib.PREC_BF16 if self.bf16 else 0
        self.T = dict(zip(MODS, T))
        self.device = torch.device(device)
        self.labels_float = labels_float
        self._drop = 0.0
        sp = spec
        D, H, nl, NC = sp.D, sp.H, sp.nl, sp.NC
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        # activations (include/mep.h MEP_PREC_BF16): bf16 on the bf16 path -- the features, unified
        # rows, attention outputs, epilogue intermediates and their gradients -- else fp32
        act = dict(dtype=torch.bfloat16 if self.bf16 else torch.float32, device=dev)
        self.act = act
        self.Ttot = sum(self.T.values())
        self.C = 3 * nl * D
        self.F = 2 * self.C
        E = 2
        # ---------------- static input buffers ([B, 2, T, d] prev/cur layout)
        # encoder-major [E, B, T, d]: each encoder's input rows are contiguous (linear in the token,
        # the fast addressing of k_wgrad); the masks keep the [B, E, T] prev/cur layout
        # bf16 feature rows padded to 8 elements (16 bytes): the bf16 kernels read column pairs
        # as dwords (k_wgrad) and 4 columns as 8 bytes (unify); the pad columns stay zero
        self.dpad = {m: (-(-d // 8) * 8 if self.bf16 else d) for m, d in zip(MODS, sp.dims)}
        self.x_in = {m: torch.zeros(E, B, self.T[m], self.dpad[m], **act) for m in MODS}
        self.m_in = {m: torch.zeros(B, E, self.T[m], **f32) for m in MODS}
        self.labels = torch.zeros(B, NC, dtype=torch.float32 if labels_float else torch.int64, device=dev)
        # dropout {seed, row0} (include/mep.h mep_epi_desc.seed), usually the runner's shared state
        self.seed_state = seed_state if seed_state is not None else torch.zeros(2, dtype=torch.int64, device=dev)
        assert self.seed_state.numel() == 2 and self.seed_state.dtype == torch.int64
        self.seed = self.seed_state[0:1]
        self.row0 = self.seed_state[1:2]
        # {loss_scale, rdrop_pairs} read by the head kernel at run time (mep_head_desc.scale): one
        # captured graph serves every data-parallel share size
        self.head_scale = torch.tensor([1.0 / B, 0.0], dtype=torch.float32, device=dev)
        self._head_scale = (1.0 / B, 0)
        # ---------------- activations
        ntok = {m: B * self.T[m] for m in MODS}
        self.ntok = ntok
        assert max(ntok.values()) < 1 << 22, 'row views are limited to 2^22 rows (csrc/common.h row_off)'
        self.U = {(e, m): torch.zeros(ntok[m], D, **act) for e in range(E) for m in MODS}
        if sp.unify_norm:
            self.Y = {(e, m): torch.zeros(ntok[m], D, **act) for e in range(E) for m in MODS}
            self.Ystat = {(e, m): torch.zeros(ntok[m], 2, **f32) for e in range(E) for m in MODS}
        self.Xcat = [torch.zeros(B, self.Ttot, self.C, **f32) for _ in range(E)]
        self.pool_fold = POOL_FOLD
        self.dXcat = None if self.pool_fold else [torch.zeros(B, self.Ttot, self.C, **f32) for _ in range(E)]
        self.pooled = [torch.zeros(B, self.F, **f32) for _ in range(E)]
        self.argmax = [torch.zeros(B, self.C, dtype=torch.int32, device=dev) for _ in range(E)]
        self.dpooled = [torch.zeros(B, self.F, **f32) for _ in range(E)]
        self.logits = torch.zeros(B, NC, **f32)
        self.row_loss = torch.zeros(B, **f32)
        self.loss = torch.zeros(1, **f32)
        self.head_stride = _lib.lib().mep_head_partial_stride(NC)
        self.head_partial = torch.zeros(B, self.head_stride, **f32)
        self.toff = {}
        t = 0
        for m in TIME_ORDER:
            self.toff[m] = t
            t += self.T[m]

        self.blocks = []
        for e in range(E):
            for j, (qm, km) in enumerate(CHAINS):
                for i in range(nl):
                    self.blocks.append(self._make_block(e, j, i, qm, km))
        self._build_descriptors()

    # ------------------------------------------------------------------ buffers per block
    def _make_block(self, e, j, i, qm, km):
        sp, B, D, H = self.spec, self.B, self.spec.D, self.spec.H
        f32 = dict(dtype=torch.float32, device=self.device)
        Tq, Tk = self.T[qm], self.T[km]
        nq, nk = B * Tq, B * Tk
        blk = dict(idx=len(self.blocks), e=e, j=j, i=i, qm=qm, km=km, Tq=Tq, Tk=Tk,
                   pre=sp.prefixes[e] + 'multimodal_blocks.%d.' % (sp.nl * j + i))
        for name in ('X', 'XP', 'Z', 'dZ', 'dXP', 'dX', 'dQ'):
            blk[name] = torch.zeros(nq, D, **self.act)
        if self.bf16 and i < sp.nl - 1:
            # bf16 copy of the block output (fp32 in the pooled tensor) for the next layer's q
            blk['Qh'] = torch.zeros(nq, D, **self.act)
        blk['estat'] = torch.zeros(nq, 2, **f32)
        blk['astat'] = torch.zeros(3 * B * H * Tq, **f32)   # (max, 1/sum) per row, then the residual rows' S_prev means
        blk['dKV'] = torch.zeros(nk, D, **self.act)
        blk['ln_partial'] = torch.zeros(cdiv(nq, 16), 2, D, **f32)   # one row per 16-token wave
        if sp.drop_p > 0:
            # the forward epilogue's dropout keep bits, read by the backward (mep_epi_desc.drop_bits)
            blk['dbits'] = torch.zeros(cdiv(nq, 16) * 2 * 64, dtype=torch.int32, device=self.device)
        if i < sp.nl - 1:
            blk['S'] = torch.zeros(B, H, Tq, Tk, **f32)
        if i >= 1:
            blk['dSprev'] = torch.zeros(B, H, Tq, Tk, **f32)
            blk['dc_partial'] = torch.zeros(_lib.attn_dc_slots(B, H, Tk), **f32)
        g = j % 3
        blk['col'] = (g * sp.nl + i) * D
        return blk

    def _out_rows(self, blk):
        e, qm = blk['e'], blk['qm']
        return rows(self.Xcat[e], blk['Tq'], self.Ttot * self.C, self.C, self.toff[qm] * self.C + blk['col'])

    def _q_rows(self, blk):
        if blk['i'] == 0:
            return crows(self.U[(blk['e'], blk['qm'])], blk['Tq'], self.spec.D)
        prev = self._blk(blk['e'], blk['j'], blk['i'] - 1)
        if 'Qh' in prev:                      # bf16 path: the previous block's bf16 output copy
            return crows(prev['Qh'], blk['Tq'], self.spec.D)
        return self._out_rows(prev)

    def _blk(self, e, j, i):
        return self.blocks[(e * 9 + j) * self.spec.nl + i]

    def _in_rows(self, e, m):
        d = self.spec.dims[MODS.index(m)]
        T = self.T[m]
        dp = self.dpad[m]
        return rows(self.x_in[m], T, T * dp, dp, e * self.B * T * dp)

    # ------------------------------------------------------------------ descriptors
    def _build_descriptors(self):
        sp, fl, B, D, H, nl, NC = self.spec, self.flat, self.B, self.spec.D, self.spec.H, self.spec.nl, self.spec.NC
        dev = self.device
        E = 2
        g = fl.gptr
        # unify
        ud = []
        for e in range(E):
            pre = sp.prefixes[e] + 'unify_dimension.'
            for m, d in zip(MODS, sp.dims):
                out = self.Y[(e, m)] if sp.unify_norm else self.U[(e, m)]
                ud.append(GemmDesc(x=self._in_rows(e, m), y=crows(out, self.T[m], D),
                                   w=fl.ptr(pre + UNIFY_NAMES[m] + '.weight'), bias=0, table=0,
                                   ntok=self.ntok[m], N=D, K=d, ldw=d, w_nt=1, accumulate=0, relu=0, alpha=1.0,
                                   bf16=(_lib.BF16_OPS | _lib.BF16_STORE) if self.bf16 else 0))
        self.d_unify, self.t_unify = make_unify(ud, dev)
        if sp.unify_norm:
            ln = []
            for e in range(E):
                pre = sp.prefixes[e] + 'unify_dimension.norm1.'
                for m in MODS:
                    T = self.T[m]
                    ln.append(LnDesc(x=crows(self.Y[(e, m)], T, D), y=crows(self.U[(e, m)], T, D),
                                     dy=Rows(), dx=Rows(), w=fl.ptr(pre + 'weight'), b=fl.ptr(pre + 'bias'),
                                     stats=self.Ystat[(e, m)].data_ptr(), partial=0, ntok=self.ntok[m], D=D,
                                     dx_accumulate=0, bf16=_lib.BF16_STORE if self.bf16 else 0))
            self.d_uln = DescArray(LnDesc, ln, dev)
        # per layer: attention + epilogue forward
        self.d_attn, self.d_epi, self.t_attn, self.t_epi, self.g_attn = [], [], [], [], []
        for i in range(nl):
            ad, ed = [], []
            for blk in (b for b in self.blocks if b['i'] == i):
                ad.append(self._attn_desc(blk))
                ed.append(self._epi_desc(blk))
            self.d_attn.append(DescArray(AttnDesc, ad, dev))
            self.d_epi.append(DescArray(EpiDesc, ed, dev))
            geo = _lib.attn_geometry(ad)
            # 16-query forward tasks (MEP_ATTN_SPLITQ) when the launch has few (b, h) units
            sq, sq_tiles = _lib.attn_fwd_splitq(ad, min_units=1024)
            if sq:
                geo = (sq_tiles, geo[1], geo[2] | sq)
            self.t_attn.append(geo[0])
            self.g_attn.append(geo)
            self.t_epi.append(_lib.epi_grid(max(B * b['Tq'] for b in self.blocks), len(ed)))
        # pool
        # (the pool's backward is formed inside the epilogue backward: no dx tensor, no launch)
        pd = [PoolDesc(x=self.Xcat[e].data_ptr(), dx=0 if self.pool_fold else self.dXcat[e].data_ptr(),
                       pooled=self.pooled[e].data_ptr(),
                       dpooled=self.dpooled[e].data_ptr(), argmax=self.argmax[e].data_ptr(),
                       B=B, T=self.Ttot, C=self.C) for e in range(E)]
        self.d_pool = DescArray(PoolDesc, pd, dev)
        self.t_pool = B * cdiv(self.C, 32)
        self.t_poolb = B * cdiv(self.Ttot, 16)
        # head
        hn = sp.head_norm
        self.head = HeadDesc(
            pooled0=self.pooled[0].data_ptr(), pooled1=self.pooled[1].data_ptr(),
            dpooled0=self.dpooled[0].data_ptr(), dpooled1=self.dpooled[1].data_ptr(),
            wc0=fl.ptr('intensity.classifier.weight'), wc1=fl.ptr('stimulation.classifier.weight'),
            trans=fl.ptr('trans'), ln_w=fl.ptr(hn + '.weight'), ln_b=fl.ptr(hn + '.bias'),
            wo=fl.ptr('out.weight'), bo=fl.ptr('out.bias'), labels=self.labels.data_ptr(),
            logits=self.logits.data_ptr(), row_loss=self.row_loss.data_ptr(),
            partial=self.head_partial.data_ptr(), B=B, F=self.F, NC=NC,
            labels_are_float=int(self.labels_float), rdrop=0, compute_grad=1, loss_scale=1.0 / B, ext_dlogits=0,
            mean_div=self.Ttot if self.pool_fold else 0,   # the fold reads dmean / T straight from dpooled
            scale=self.head_scale.data_ptr())
        # per-modality gradient sums
        sd = []
        self.dU = {}
        for e in range(E):
            for m in MODS:
                T = self.T[m]
                self.dU[(e, m)] = torch.zeros(self.ntok[m], D, **self.act)
                srcs = [crows(self._blk(e, j, 0)['dQ'], T, D) for j, (qm, km) in enumerate(CHAINS) if qm == m]
                srcs += [crows(self._blk(e, j, i)['dKV'], T, D) for j, (qm, km) in enumerate(CHAINS) if km == m
                         for i in range(nl)]
                assert len(srcs) <= _lib.SUM_MAX_SRC
                arr = (Rows * _lib.SUM_MAX_SRC)(*srcs)
                sd.append(SumDesc(src=arr, out=crows(self.dU[(e, m)], T, D), n_src=len(srcs),
                                  ntok=self.ntok[m], D=D, accumulate=_lib.SUM_BF16 if self.bf16 else 0))
        self.d_sum = DescArray(SumDesc, sd, dev)
        self.t_sum = min(1024, max(cdiv(self.ntok[m] * D // 4, 256) for m in MODS))
        # backward per layer
        self.d_epib, self.d_attnb, self.t_attnb, self.f_attnb = [], [], [], []
        for i in range(nl):
            eb, ab = [], []
            for blk in (b for b in self.blocks if b['i'] == i):
                eb.append(self._epi_bwd_desc(blk))
                ab.append(self._attn_bwd_desc(blk))
            self.d_epib.append(DescArray(EpiBwdDesc, eb, dev))
            self.d_attnb.append(DescArray(AttnBwdDesc, ab, dev))
            self.t_attnb.append(self.g_attn[i][1])
            self.f_attnb.append(_lib.attn_bwd_flags(ab))
        if sp.unify_norm:
            self.dY = {k: torch.zeros_like(v) for k, v in self.dU.items()}
            tiles = {m: cdiv(self.ntok[m], 64) for m in MODS}
            self.uln_partial = [torch.zeros(sum(tiles.values()), 2, D, dtype=torch.float32, device=dev)
                                for _ in range(E)]
            lb = []
            for e in range(E):
                pre = sp.prefixes[e] + 'unify_dimension.norm1.'
                r0 = 0
                for m in MODS:
                    T = self.T[m]
                    lb.append(LnDesc(x=crows(self.Y[(e, m)], T, D), y=Rows(), dy=crows(self.dU[(e, m)], T, D),
                                     dx=crows(self.dY[(e, m)], T, D), w=fl.ptr(pre + 'weight'), b=0,
                                     stats=self.Ystat[(e, m)].data_ptr(),
                                     partial=self.uln_partial[e].data_ptr() + 4 * r0 * 2 * D,
                                     ntok=self.ntok[m], D=D, dx_accumulate=0,
                                     bf16=_lib.BF16_STORE if self.bf16 else 0))
                    r0 += tiles[m]
            self.d_ulnb = DescArray(LnDesc, lb, dev)
        self._build_grad_descriptors()

    def _attn_desc(self, blk):
        sp, fl, D = self.spec, self.flat, self.spec.D
        e, km = blk['e'], blk['km']
        kv = crows(self.U[(e, km)], blk['Tk'], D)
        Tk = self.T[km]
        prev = self._blk(e, blk['j'], blk['i'] - 1) if blk['i'] > 0 else None
        return AttnDesc(q=self._q_rows(blk), k=kv, v=kv, x=crows(blk['X'], blk['Tq'], D),
                        mask=self.m_in[km].data_ptr() + 4 * e * Tk, mask_sB=2 * Tk,
                        s_prev=prev['S'].data_ptr() if prev is not None else 0,
                        c=fl.ptr(blk['pre'] + 'c'), s_out=blk['S'].data_ptr() if 'S' in blk else 0,
                        stats=blk['astat'].data_ptr(), B=self.B, H=sp.H, Tq=blk['Tq'], Tk=Tk)

    def _epi_desc(self, blk):
        sp, fl, D = self.spec, self.flat, self.spec.D
        Tq = blk['Tq']
        stream_id = blk['idx']
        return EpiDesc(q=self._q_rows(blk), x=crows(blk['X'], Tq, D), xp=crows(blk['XP'], Tq, D),
                       z=crows(blk['Z'], Tq, D), out=self._out_rows(blk),
                       wp=fl.ptr(blk['pre'] + 'proj.weight'), wm=fl.ptr(blk['pre'] + 'minus.weight'),
                       ln_w=fl.ptr(blk['pre'] + sp.block_norm + '.weight'),
                       ln_b=fl.ptr(blk['pre'] + sp.block_norm + '.bias'),
                       stats=blk['estat'].data_ptr(), seed=self.seed_state.data_ptr(),
                       ntok=self.B * Tq, D=D, drop_p=self._drop, drop_stream=stream_id,
                       out_h=crows(blk['Qh'], Tq, D) if 'Qh' in blk else Rows(),
                       drop_bits=blk['dbits'].data_ptr() if 'dbits' in blk else 0)

    def _epi_bwd_desc(self, blk):
        D, Tq = self.spec.D, blk['Tq']
        nxt = self._blk(blk['e'], blk['j'], blk['i'] + 1) if blk['i'] < self.spec.nl - 1 else None
        e = blk['e']
        # upstream gradient: the mean+max pool's backward of this block's slice of Xcat (formed in
        # the kernel from dpooled / argmax) + the next layer's dq
        if self.pool_fold:
            up = dict(dout=Rows(), pool_T=-self.Ttot, pool_dpooled=self.dpooled[e].data_ptr(),
                      pool_argmax=self.argmax[e].data_ptr(), pool_C=self.C, pool_Tq=Tq,
                      pool_t0=self.toff[blk['qm']], pool_col=blk['col'])
        else:
            up = dict(dout=rows(self.dXcat[e], Tq, self.Ttot * self.C, self.C,
                                self.toff[blk['qm']] * self.C + blk['col']))
        return EpiBwdDesc(f=self._epi_desc(blk),
                          dout2=crows(nxt['dQ'], Tq, D) if nxt is not None else Rows(),
                          dz=crows(blk['dZ'], Tq, D), dxp=crows(blk['dXP'], Tq, D), dx=crows(blk['dX'], Tq, D),
                          dq=crows(blk['dQ'], Tq, D), ln_partial=blk['ln_partial'].data_ptr(), dq_accumulate=0,
                          **up)

    def _attn_bwd_desc(self, blk):
        D = self.spec.D
        nxt = self._blk(blk['e'], blk['j'], blk['i'] + 1) if blk['i'] < self.spec.nl - 1 else None
        dkv = crows(blk['dKV'], blk['Tk'], D)
        return AttnBwdDesc(f=self._attn_desc(blk), dx=crows(blk['dX'], blk['Tq'], D),
                           dq=crows(blk['dQ'], blk['Tq'], D), dk=dkv, dv=dkv,
                           ds_next=nxt['dSprev'].data_ptr() if nxt is not None else 0,
                           ds_prev=blk['dSprev'].data_ptr() if 'dSprev' in blk else 0,
                           dc_partial=blk['dc_partial'].data_ptr() if 'dc_partial' in blk else 0)

    def _build_grad_descriptors(self):
        """Descriptors of the launches that write into the flat gradient buffer."""
        sp, fl, D = self.spec, self.flat, self.spec.D
        dev = self.device
        g = fl.gptr
        items = []
        for blk in self.blocks:
            Tq, nq, pre = blk['Tq'], self.B * blk['Tq'], blk['pre']
            items.append((crows(blk['dXP'], Tq, D), D, nq, [(crows(blk['X'], Tq, D), D, g(pre + 'proj.weight'), D)]))
            items.append((crows(blk['dZ'], Tq, D), D, nq, [(self._q_rows(blk), D, g(pre + 'minus.weight'), 2 * D),
                                                           (crows(blk['XP'], Tq, D), D,
                                                            g(pre + 'minus.weight') + 4 * D, 2 * D)]))
        for e in range(2):
            pre = sp.prefixes[e] + 'unify_dimension.'
            for m, d in zip(MODS, sp.dims):
                src = self.dY[(e, m)] if sp.unify_norm else self.dU[(e, m)]
                items.append((crows(src, self.T[m], D), D, self.ntok[m],
                              [(self._in_rows(e, m), d, g(pre + UNIFY_NAMES[m] + '.weight'), d)]))
        self._wgrad_items = items
        self._n_block_items = 2 * len(self.blocks)   # items[:n]: block weights (bucket A)
        self.wg_partial, self.d_wgrad, self.t_wgrad, self.t_wgred = make_wgrad(items, dev, bf16=self.bf16)
        # column sums: block LayerNorms, residual coefficients, Ren unify LayerNorm
        cs, self._colsum_a, self._colsum_b = [], [], []
        for blk in self.blocks:
            nt = blk['ln_partial'].shape[0]
            base = blk['ln_partial'].data_ptr()
            nm = blk['pre'] + sp.block_norm
            for c_ in (ColsumDesc(partial=base, out=g(nm + '.weight'), n_rows=nt, n_cols=D, ld=2 * D, accumulate=0),
                       ColsumDesc(partial=base + 4 * D, out=g(nm + '.bias'), n_rows=nt, n_cols=D, ld=2 * D,
                                  accumulate=0)):
                cs.append(c_)
                self._colsum_a.append(c_)
            if 'dc_partial' in blk:
                c_ = ColsumDesc(partial=blk['dc_partial'].data_ptr(), out=g(blk['pre'] + 'c'),
                                n_rows=blk['dc_partial'].numel(), n_cols=1, ld=1, accumulate=0)
                cs.append(c_)
                self._colsum_b.append(c_)
        if sp.unify_norm:
            for e in range(2):
                pre = sp.prefixes[e] + 'unify_dimension.norm1.'
                p = self.uln_partial[e]
                for c_ in (ColsumDesc(partial=p.data_ptr(), out=g(pre + 'weight'), n_rows=p.shape[0], n_cols=D,
                                      ld=2 * D, accumulate=0),
                           ColsumDesc(partial=p.data_ptr() + 4 * D, out=g(pre + 'bias'), n_rows=p.shape[0],
                                      n_cols=D, ld=2 * D, accumulate=0)):
                    cs.append(c_)
                    self._colsum_b.append(c_)
        self.d_colsum = DescArray(ColsumDesc, cs, dev)
        self.t_colsum = cdiv(D, 32)
        hn = sp.head_norm
        self.head_grads = (g('trans'), g(hn + '.weight'), g(hn + '.bias'), g('out.weight'), g('out.bias'),
                           g('intensity.classifier.weight'), g('stimulation.classifier.weight'),
                           self.loss.data_ptr())
        self.d_losssum = DescArray(ColsumDesc, [ColsumDesc(partial=self.row_loss.data_ptr(), out=self.loss.data_ptr(),
                                                           n_rows=self.B, n_cols=1, ld=1, accumulate=0)], dev)
        self.redmap = reduce_map(self.d_wgrad, self.d_colsum, self.head, dev)

    # ------------------------------------------------------------------ execution
    def set_inputs(self, l, v, a, lm, vm, am, labels=None):
        with torch.no_grad():
            for m, x, mk in (('l', l, lm), ('v', v, vm), ('a', a, am)):
                if isinstance(x, (tuple, list)):      # (prev, cur) pair of [B, T, d]
                    for e in range(2):
                        self.x_in[m][e, ..., :x[e].shape[-1]].copy_(x[e])
                        self.m_in[m][:, e].copy_(mk[e])
                else:                                 # [B, 2, T, d]
                    self.x_in[m][..., :x.shape[-1]].copy_(x.transpose(0, 1))
                    self.m_in[m].copy_(mk)
            if labels is not None:
                self.labels.copy_(labels)

    def set_global_rows(self, n):
        """Scale the fused loss for a data-parallel share (mep_amd.dp): the circle loss by
        1/n (the rank's part of the global-batch mean) and the R-Drop KL batchmean by n/2 global
        pairs; None restores the local mean (1/B, B/2).  The values live in a device buffer the
        head kernel reads at run time, so a captured graph replays any share unchanged."""
        rows = self.B if n is None else int(n)
        val = (1.0 / rows, 0 if n is None else rows // 2)
        if val != self._head_scale:          # two device fills, no host sync
            self.head_scale[0].fill_(val[0])
            self.head_scale[1].fill_(float(val[1]))
            self._head_scale = val
        self.head.loss_scale, self.head.rdrop_pairs = val
        return rows

    def set_row0(self, row0):
        """Global index of this batch's first row (data-parallel share): the dropout masks of
        local row b are the full batch's masks of row row0 + b.  The slot lives in the model's
        seed_state (shared by its plans), so the value last written is kept on that tensor with
        the tensor's version counter: an unchanged row0 costs no device fill per step, and any
        other in-place write of seed_state through torch (zero_, copy_ from a saved state, a test
        poking it) bumps the version and forces the fill.  mep_seed_advance writes seed[0] only."""
        row0 = int(row0)
        if getattr(self.seed_state, '_mep_row0', None) != (row0, self.seed_state._version):
            self.row0.fill_(row0)
            self.seed_state._mep_row0 = (row0, self.seed_state._version)

    def set_dropout(self, p):
        """Dropout probability of the block epilogues (Ren-MME DROP at train time, 0 in eval).
        Descriptor bytes are rewritten in place so captured graphs see the new value."""
        p = float(p)
        if p == self._drop:
            return
        self._drop = p
        for i in range(self.spec.nl):
            blks = [b for b in self.blocks if b['i'] == i]
            for arr, items in ((self.d_epi[i], [self._epi_desc(b) for b in blks]),
                               (self.d_epib[i], [self._epi_bwd_desc(b) for b in blks])):
                host = (arr.struct * arr.n)(*items)
                arr.dev.copy_(torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8))

    def forward(self, grad=True, rdrop=False, stream=None):
        """Encoder forward + pool + fused head.  The head always produces logits and the per-row
        loss (row_loss, already scaled by 1/B); grad=True also runs the head backward
        (dpooled + head parameter partials) inside the same launch."""
        sp, nl = self.spec, self.spec.nl
        _lib.gemm('mep_unify', self.d_unify, self.t_unify, stream, prec=self.prec)
        if sp.unify_norm:
            launch('mep_layernorm_fwd', self.d_uln, cdiv(max(self.ntok.values()), 4), stream)
        for i in range(nl):
            launch('mep_attn_fwd', self.d_attn[i], self.t_attn[i], stream, threads=self.g_attn[i][2] | self.prec)
            launch('mep_block_epi_fwd', self.d_epi[i], self.t_epi[i], stream, threads=sp.D | self.prec)
        launch('mep_pool_fwd', self.d_pool, self.t_pool, stream)
        self.head.compute_grad = int(grad)
        self.head.rdrop = int(rdrop)
        self.head.ext_dlogits = 0
        _lib.call('mep_head_fwd_bwd', ctypes.byref(self.head), stream=stream)

    def backward(self, ext_dlogits=None, stream=None):
        """Backward from the fused-loss head partials, or from external dlogits [B, NC].
        Writes every parameter gradient into the flat gradient buffer (flat.grad) and the batch
        loss into self.loss."""
        sp, nl = self.spec, self.spec.nl
        if ext_dlogits is not None:
            self.head.compute_grad = 1
            self.head.ext_dlogits = ext_dlogits.data_ptr()
            _lib.call('mep_head_fwd_bwd', ctypes.byref(self.head), stream=stream)
            self.head.ext_dlogits = 0
        if not self.pool_fold:
            launch("mep_pool_bwd", self.d_pool, self.t_poolb, stream)
        for i in reversed(range(nl)):
            launch('mep_block_epi_bwd', self.d_epib[i], self.t_epi[i], stream, threads=sp.D | self.prec)
            launch('mep_attn_bwd', self.d_attnb[i], self.t_attnb[i], stream, threads=self.f_attnb[i] | self.prec)
        launch('mep_sum_rows', self.d_sum, self.t_sum, stream)
        if sp.unify_norm:
            launch('mep_layernorm_bwd', self.d_ulnb, cdiv(max(self.ntok.values()), 64), stream)
        launch('mep_wgrad', self.d_wgrad, self.t_wgrad, stream)
        # weight-gradient split sums, LayerNorm / residual-coefficient column sums and the head
        # parameter sums: one launch over the real jobs only
        reduce_mapped(self.d_wgrad, self.d_colsum, self.head, self.head_grads, _norm_args(self), self.redmap, stream)

    norm_fold = None   # (optimizer workspace, step, hyper) pointers: the clip's norm pass folded into the reduction

    def reduce_grid(self):
        """blocks of the backward's mep_reduce_grads launch (the optimizer's folded norm partials)"""
        return reduce_blocks(self.d_wgrad, self.d_colsum, self.head, self.redmap)

    def advance_seed(self, stream=None):
        _lib.call('mep_seed_advance', ctypes.c_void_p(self.seed.data_ptr()), stream=stream)

    def _build_buckets(self):
        """Weight-gradient and reduction launches split by gradient bucket (FlatParams.split):
        A = block weights + block LayerNorms + fusion head, B = unify weights (+ unify LayerNorm)
        + residual coefficients.  Both launches keep the fused launch's token chunk, so every
        gradient is the same sum in the same order, bit for bit."""
        if getattr(self, '_buckets', None) is not None:
            return
        dev, items, nb = self.device, self._wgrad_items, self._n_block_items
        if WG_BALANCE:   # the one-launch form's segment counts, the B items renumbered from 0
            cnt = wgrad_counts(items, wg_target(self.bf16), bf16=self.bf16)
            wa = make_wgrad(items[:nb], dev, bf16=self.bf16, counts={u: k for u, k in cnt.items() if u[0] < nb})
            wb = make_wgrad(items[nb:], dev, bf16=self.bf16,
                            counts={(i - nb, cg): k for (i, cg), k in cnt.items() if i >= nb})
        else:
            tps = wgrad_chunk(items, wg_target(self.bf16), bf16=self.bf16)
            wa = make_wgrad(items[:nb], dev, tok_per_split=tps, bf16=self.bf16)
            wb = make_wgrad(items[nb:], dev, tok_per_split=tps, bf16=self.bf16)
        ca = DescArray(ColsumDesc, self._colsum_a, dev)
        cb = DescArray(ColsumDesc, self._colsum_b, dev)
        self._check_bucket_ranges(wa[1], wb[1], ca, cb)
        self._buckets = (wa, wb, ca, cb)
        self._bucket_maps = (reduce_map(wa[1], ca, self.head, dev), reduce_map(wb[1], cb, None, dev))

    def _check_bucket_ranges(self, wa, wb, ca, cb):
        """Bucket membership is defined twice -- by parameter name (TriModalSpec.bucket_a, which
        orders the flat buffer) and by descriptor order (_n_block_items, _colsum_a / _colsum_b) --
        so check on the host that every gradient byte bucket A's launches write lies in
        flat.grad[:split] and every byte bucket B's write lies in flat.grad[split:n_grad]: a write
        outside its bucket would race the side-stream all-reduce (engine.py)."""
        fl = self.flat
        g0 = fl.grad.data_ptr()
        lo_hi = {'A': (g0, g0 + 4 * fl.split), 'B': (g0 + 4 * fl.split, g0 + 4 * fl.n_grad)}

        def extents(warr, carr):
            for d in warr.items:
                for b in range(d.n_b):
                    rows_, cols_ = (d.kb[b], d.N) if d.out_trans else (d.N, d.kb[b])
                    yield d.out[b], d.out[b] + 4 * ((rows_ - 1) * d.ldo[b] + cols_)
            for c in carr.items:
                yield c.out, c.out + 4 * c.n_cols
        head = [p for p in self.head_grads[:-1]]          # the last entry is the loss, not a gradient
        for name, warr, carr, extra in (('A', wa, ca, head), ('B', wb, cb, [])):
            lo, hi = lo_hi[name]
            for a, b in list(extents(warr, carr)) + [(p, p + 4) for p in extra]:
                assert lo <= a and b <= hi, ('gradient write [%#x, %#x) outside bucket %s [%#x, %#x)'
                                             % (a, b, name, lo, hi))

    def backward_bucketed(self, bucket_a_done, ext_dlogits=None, stream=None):
        """backward() with the gradient reductions split by bucket: bucket A's gradients are
        complete (and bucket_a_done() is called, e.g. to start its all-reduce on a side stream)
        right after the last epilogue backward, before the last attention backward; bucket B's
        at the end."""
        sp, nl = self.spec, self.spec.nl
        self._build_buckets()
        (pa, da, ta, ra), (pb, db, tb, rb), ca, cb = self._buckets
        if ext_dlogits is not None:
            self.head.compute_grad = 1
            self.head.ext_dlogits = ext_dlogits.data_ptr()
            _lib.call('mep_head_fwd_bwd', ctypes.byref(self.head), stream=stream)
            self.head.ext_dlogits = 0
        if not self.pool_fold:
            launch("mep_pool_bwd", self.d_pool, self.t_poolb, stream)
        for i in reversed(range(nl)):
            launch('mep_block_epi_bwd', self.d_epib[i], self.t_epi[i], stream, threads=sp.D | self.prec)
            if i == 0:
                launch('mep_wgrad', da, ta, stream)
                reduce_mapped(da, ca, self.head, self.head_grads, (None, None, None), self._bucket_maps[0], stream)
                bucket_a_done()
            launch('mep_attn_bwd', self.d_attnb[i], self.t_attnb[i], stream, threads=self.f_attnb[i] | self.prec)
        launch('mep_sum_rows', self.d_sum, self.t_sum, stream)
        if sp.unify_norm:
            launch('mep_layernorm_bwd', self.d_ulnb, cdiv(max(self.ntok.values()), 64), stream)
        launch('mep_wgrad', db, tb, stream)
        reduce_mapped(db, cb, None, None, (None, None, None), self._bucket_maps[1], stream)

    def loss_only(self, stream=None):
        """Batch loss (sum of the scaled per-row losses) without the backward."""
        launch('mep_colsum', self.d_losssum, 1, stream)
