"""Algorithmic FLOPs and HBM bytes per launch of a TriModalPlan step.

"Algorithmic" = the minimum the launch must move: every DISTINCT input tensor read once, every
output written once, no recomputation (the attention backward's recomputed S / dP are not
counted).  fp32 (4 B).  Inputs shared by several blocks of one launch count once (round 6): a
modality's unified features are the queries of three chains and the keys / values of three more,
so the attention launches read each of them once, and L2 / the Infinity Cache serve the rest.
Per attention-block instance (batch row b, block j), with n_kv = 1 (k is v):
  fwd flops = 4*Tq*Tk*D;  bytes = 4*(Tq*D (x) + [q, kv rows once per distinct tensor]) + 4*Tk
          + 8*H*Tq + 4*H*Tq*Tk*(r_in + r_out)
  bwd flops = 10*Tq*Tk*D; bytes = 4*(Tq*D*(x, dx, dq r+w) + Tk*D*dkv + [q, kv once per distinct
          tensor]) + 4*Tk + 8*H*Tq (+ S_prev, ds_next reads, ds_prev write when chained)
VALU issue floor (valu_floor): a wave64 VALU instruction occupies its SIMD for 4 cycles, so a
launch issuing N of them needs at least 4 N / (1,024 SIMDs x 2.4 GHz); N per dispatch comes from
the committed SQ_INSTS_VALU counter pass of the workload (profiles/r*_counters_*.json).
Peaks (MI355X_MICROARCH.md): HBM 8.0 TB/s; fp32 MFMA (= vector rate) 157.3 TFLOP/s; bf16 MFMA
2.5 PFLOP/s dense.  Kernels whose fp32 products run as bf16 parts (split.h) are priced against the
bf16 peak divided by the bf16 products per fp32 product (compute_peak): six for the 3-part x 3-part
kernels (weight gradients, tiled token GEMM, attention forward scores and P.V, the D <= 96
epilogue forward): 2.5 P / 6 = 417 TFLOP/s; five for the 2-part-weight x 3-part-activation
products (D = 128 epilogues; Wm^T of the single-phase D <= 96 epilogue backward, 2/3 of its
flops, the 3-part Wp^T the rest); four for the attention backward's S, dP, dV, dK and three for
its dQ: 658 TFLOP/s.  The realformer token GEMMs and epilogues: on the wave-tiled kernels
(mep_wgemm, mep_rfw_epi_*: six products) 417 TFLOP/s; on the LDS-tiled ones (MEP_RFW=0: mep_gemm,
mep_rf_epi_*) f32 MFMA, 157 TF.
bf16 path (MEP_PREC_BF16): one bf16 product per product, every matrix kernel priced at the bf16
peak; the activations (features, unified rows, attention outputs, xp / z and their gradients) are
stored as bf16, so their bytes count 2 per element (include/mep.h); block outputs (the pooled
tensor), scores, statistics and parameters stay 4.
"""
from . import _lib
from .trimodal import MODS

HBM_PEAK = 8.0e12
SIMDS, CLOCK, VALU_CYCLES = 1024, 2.4e9, 4          # 256 CUs x 4 SIMDs; wave64 VALU issue cycles
F32_PEAK = 157.3e12
BF16_PEAK = 2.5e15
# fp32 path (csrc/attn.hip): the forward's scores and P.V take six bf16 products each (3-part
# splits, MEP_FWD_PVSPLIT = 2); the backward's S, dP, dV, dK four (2-part) and dQ three: ideal
# time per 2*Tq*Tk*D-flop contraction at the bf16 peak / products
ATTN_FWD_PEAK = 4.0 / (2.0 * (6 + 6) / BF16_PEAK)
ATTN_BWD_PEAK = 10.0 / (2.0 * (4 + 4 + 4 + 4 + 3) / BF16_PEAK)
COMPUTE_PEAK = {'mep_block_epi_fwd': BF16_PEAK / 6, 'mep_block_epi_bwd': BF16_PEAK / 6, 'mep_wgrad': BF16_PEAK / 6,
                'mep_tgemm': BF16_PEAK / 6, 'mep_wgemm': BF16_PEAK / 6, 'mep_wgemm_ws': BF16_PEAK / 6, 'mep_wgemm_sum': BF16_PEAK / 6, 'mep_rfw_front': BF16_PEAK / 6,
                'mep_rfw_epi_fwd': BF16_PEAK / 6, 'mep_rfw_epi_bwd': BF16_PEAK / 6,
                'mep_attn_fwd': ATTN_FWD_PEAK, 'mep_attn_bwd': ATTN_BWD_PEAK}


def compute_peak(name, D=None, bf16=False):
    """The compute peak a launch is priced against (csrc/block.hip: MEP_EPI_SPLIT128 and
    MEP_EPI_ONE_BWD, both on by default, decide the epilogues' product counts)."""
    if bf16:
        return BF16_PEAK
    if name == 'mep_block_epi_fwd' and D == 128:
        return BF16_PEAK / 5
    if name == 'mep_block_epi_bwd' and D is not None and D <= 128:
        # D = 128: five products; D <= 96 single phase: Wm^T (2/3 of the flops) five, Wp^T six
        return BF16_PEAK / 5 if D == 128 else 1.0 / ((2.0 / 3.0) * 5 / BF16_PEAK + (1.0 / 3.0) * 6 / BF16_PEAK)
    return COMPUTE_PEAK.get(name, F32_PEAK)


def launch_costs(plan):
    """{launch name: (flops, bytes)} for one eager training step of the plan (summed over the
    layers when a launch repeats)."""
    if hasattr(plan, 'rfw') or not hasattr(plan, 'Xcat'):      # RealformerPlan (chain or State_Transfer)
        return rf_launch_costs(plan)
    sp, B = plan.spec, plan.B
    D, H = sp.D, sp.H
    a = 2 if getattr(plan, 'bf16', False) else 4     # bytes per activation element
    out = {}
    UNIFY = _lib.gemm_launcher('mep_unify', plan.d_unify)

    def add(name, f, b):
        f0, b0 = out.get(name, (0, 0))
        out[name] = (f0 + f, b0 + b)

    for e in range(2):
        for m, d in zip(MODS, sp.dims):
            n = plan.ntok[m]
            add(UNIFY, 2 * n * D * d, a * (n * d + n * D) + 4 * D * d)
    for name, (f, b) in attn_costs(plan, a).items():
        add(name, f, b)
    shared_q = set()
    for blk in plan.blocks:
        Tq, Tk = blk['Tq'], blk['Tk']
        n = B * Tq
        # reads q, x; writes xp, z (activations) and out (the pooled tensor, fp32) [+ its bf16
        # copy for the next layer's q]
        out_h = a if (a == 2 and blk['i'] < sp.nl - 1) else 0
        add('mep_block_epi_fwd', 2 * n * D * 3 * D + 8 * n * D, a * n * D * 4 + (4 + out_h) * n * D + 8 * n + 4 * 3 * D * D + 8 * D)
        # upstream gradient formed from this block's dpooled / argmax slices (B x 3D), not read
        # as [n, D] rows (the pool backward is folded into this launch)
        add('mep_block_epi_bwd', 2 * n * D * 3 * D + 10 * n * D,
            a * n * D * 6 + 8 * n + 4 * 3 * D * D + 4 * (n // 64 + 1) * 2 * D + 4 * B * 3 * D)
        # dXP, X, dZ, XP per block; q (layer 0: the query modality's unified rows, shared by its
        # three chains) once per distinct tensor
        q_key = (blk['e'], blk['qm']) if blk['i'] == 0 else id(blk)
        add('mep_wgrad', 2 * n * D * 3 * D, a * n * D * (4 + (q_key not in shared_q)))
        shared_q.add(q_key)
    for e in range(2):
        for m, d in zip(MODS, sp.dims):
            n = plan.ntok[m]
            add('mep_wgrad', 2 * n * D * d, a * n * (D + d))
    for e in range(2):
        add('mep_pool_fwd', B * plan.Ttot * plan.C, 4 * B * (plan.Ttot * plan.C + 2 * plan.C) + 4 * B * plan.C)
        for m in MODS:                       # dU = the dQ / dKV rows of every block reading m
            n = plan.ntok[m]
            srcs = sum(1 for b in plan.blocks if b['i'] == 0 and b['qm'] == m) // 2 + \
                sum(1 for b in plan.blocks if b['km'] == m) // 2
            add('mep_sum_rows', srcs * n * D, a * n * D * (srcs + 1))
    return out


def _distinct(views):
    """bytes of the distinct tensors among (ptr, bytes) views (a tensor read by several
    descriptors of one launch counts once)"""
    seen = {}
    for p, nb in views:
        seen[p] = max(seen.get(p, 0), nb)
    return sum(seen.values())


def attn_costs(plan, a):
    """(flops, algorithmic bytes) of the attention launches of a plan, from its descriptors:
    q / k / v rows and masks once per distinct tensor, per-block outputs, statistics and score
    tensors once per descriptor (a: bytes per activation element)."""
    out = {}
    D = plan.spec.D
    fwd = [d for arr in plan.d_attn for d in arr.items]
    bwd = [d for arr in plan.d_attnb for d in arr.items]

    def rows(v, B):
        return v.ptr, a * B * v.T * D

    def fwd_bytes(d):
        s_bytes = 4 * d.H * d.Tq * d.Tk * d.B
        stat = 12 if d.s_prev else 8   # (max, 1/sum) per row, + the S_prev mean (mep.h, ABI 6)
        return (a * d.B * d.Tq * D + stat * d.B * d.H * d.Tq +
                s_bytes * ((1 if d.s_prev else 0) + (1 if d.s_out else 0)))
    f = sum(4 * d.B * d.Tq * d.Tk * D for d in fwd)
    shared = _distinct([rows(d.q, d.B) for d in fwd] + [rows(d.k, d.B) for d in fwd] + [rows(d.v, d.B) for d in fwd] +
                       [(d.mask, 4 * d.B * d.Tk) for d in fwd])
    out['mep_attn_fwd'] = (f, shared + sum(fwd_bytes(d) for d in fwd))

    def bwd_bytes(bd):
        d = bd.f
        s_bytes = 4 * d.H * d.Tq * d.Tk * d.B
        dkv = 1 if bd.dk.ptr == bd.dv.ptr else 2
        chained = s_bytes * ((1 if bd.ds_next else 0) + (2 if d.s_prev else 0))
        stat = 12 if d.s_prev else 8
        return a * d.B * (4 * d.Tq * D + dkv * d.Tk * D) + stat * d.B * d.H * d.Tq + chained
    f = sum(10 * bd.f.B * bd.f.Tq * bd.f.Tk * D for bd in bwd)
    shared = _distinct([rows(bd.f.q, bd.f.B) for bd in bwd] + [rows(bd.f.k, bd.f.B) for bd in bwd] +
                       [rows(bd.f.v, bd.f.B) for bd in bwd] + [(bd.f.mask, 4 * bd.f.B * bd.f.Tk) for bd in bwd])
    out['mep_attn_bwd'] = (f, shared + sum(bwd_bytes(bd) for bd in bwd))
    return out


def rf_launch_costs(plan):
    """Every priced launch of a realformer plan (RealformerPlan, others/realformer.py:133-318): the
    token GEMMs (Conv1d unify + position table, w_qkv, the backward's input-gradient products),
    attention (K and V separately projected: n_kv = 2, residual scores carried between the chain's
    layers), the fused RealFormer epilogue (proj, ReZero residual, LN1, FFN, LN2) forward and
    backward, the weight gradients and the per-modality gradient sums."""
    sp, R = plan.spec, plan.R
    D, H, FD = sp.D, sp.H, sp.FD
    out = {}

    def add(name, f, b):
        f0, b0 = out.get(name, (0, 0))
        out[name] = (f0 + f, b0 + b)

    rfw = getattr(plan, 'rfw', False)
    # the launcher of each token-GEMM group (rfw: mep_wgemm_ws for large launches, else mep_wgemm)
    G_UNIFY, G_PROJ = plan.gemm_launcher(plan.d_unify), plan.gemm_launcher(plan.d_proj)
    G_IN = plan.gemm_launcher(plan.d_ingrad_all) if rfw else G_PROJ
    isum = getattr(plan, 'd_isum', None) is not None
    if isum:    # mep_wgemm_sum: the input-gradient GEMMs write their per-modality sums only
        G_IN = 'mep_wgemm_sum'
    front = bool(getattr(plan, 'front', None))
    if front:   # mep_rfw_front: the projections read U from registers, not HBM
        G_UNIFY = G_PROJ = 'mep_rfw_front'
    EPI_F, EPI_B = ('mep_rfw_epi_fwd', 'mep_rfw_epi_bwd') if rfw else ('mep_rf_epi_fwd', 'mep_rf_epi_bwd')

    def gemm(name, ntok, N, K, accumulate=False, table=0, x_read=True):
        add(name, 2 * ntok * N * K, 4 * (ntok * K * x_read + ntok * N * (2 if accumulate else 1) + N * K + table))

    for m in sp.mods:                                          # unify + position table
        gemm(G_UNIFY, plan.ntok[m], D, sp.dims[m], table=plan.T[m] * D)
    for blk in plan.blocks:
        Tq, Tk, nq, nk = blk['Tq'], blk['Tk'], blk['nq'], blk['nk']
        gemm(G_PROJ, nk, 2 * D, D, x_read=not front)           # [K | V] = U [W_k; W_v]^T
        if rfw and blk['i'] > 0:
            # fused into the previous layer's epilogue launches (q = that layer's output):
            # Q = q W_q^T after its LN2, dq_in += dQ W_q before its LN2 backward
            add(EPI_F, 2 * nq * D * D, 4 * nq * D + 4 * D * D)
            add(EPI_B, 2 * nq * D * D, 4 * nq * D + 4 * D * D)
        else:
            gemm(G_PROJ, nq, D, D, x_read=not front)           # Q = q W_q^T
            gemm(G_IN, nq, D, D, accumulate=True)              # dq_in += dQ W_q
        gemm(G_IN, nk, D, 2 * D)                               # dkv_in = [dK | dV] [W_k; W_v]
        if isum:   # (no per-source row writes: one sum row per token, below)
            add(G_IN, 0, -4 * (nk * D + (nq * D if blk['i'] == 0 else 0)))
        w = 4 * (D * D + 2 * D * FD + 2 * D + FD + 4 * D)      # Wp, W1, W2, biases, LN weights
        # forward: reads q, x; writes xp, h, f1, f, out and 4 stats per token
        add(EPI_F, 2 * nq * (D * D + 2 * D * FD), 4 * nq * (7 * D + FD + 4) + w)
        # backward: reads dout, h, f, f1, q, xp, stats; writes df, df1, dxp, dx, dq
        add(EPI_B, 2 * nq * (D * D + 2 * D * FD), 4 * nq * (10 * D + 2 * FD + 4) + w)
        # weight gradients: W_q, [W_k; W_v], Wp, W1, W2
        for (n, N, K) in ((nq, D, D), (nk, D, 2 * D), (nq, D, D), (nq, D, FD), (nq, D, FD)):
            add('mep_wgrad', 2 * n * N * K, 4 * n * (N + K))
    for name, (f, b) in attn_costs(plan, 4).items():
        add(name, f, b)
    if rfw:
        # mep_wsplit: every pre-split weight read once (fp32) and its three bf16 parts written
        nw = sum(d.nrows * d.K for d in plan.d_wsplit.items)
        add('mep_wsplit', 0, nw * (4 + 6))
    for m in sp.mods:
        n = plan.ntok[m]
        add('mep_wgrad', 2 * n * D * sp.dims[m], 4 * n * (D + sp.dims[m]))
        srcs = sum(1 for (qm, km) in sp.chains if qm == m) + sum(sp.nl for (qm, km) in sp.chains if km == m)
        if isum:
            add(G_IN, srcs * n * D, 4 * n * D)
        else:
            add('mep_sum_rows', srcs * n * D, 4 * n * D * (srcs + 1))
    return out


def valu_floor(valu_insts):
    """seconds the VALU issue of `valu_insts` wave64 instructions takes with every SIMD busy"""
    return VALU_CYCLES * valu_insts / (SIMDS * CLOCK)


def roofline_entry(name, flops, nbytes, seconds, bf16=False, D=None, valu=None):
    """The bench's roofline object for one kernel: bound = the larger of the HBM and matrix-core
    ideal times (the contract's two bounds).  valu = (VALU instructions per launch, source): the
    VALU issue floor beside them (`valu`), and `limiter` names whichever of the three floors is
    largest -- 'valu' for kernels whose instruction issue, not bytes or matrix flops, sets the
    floor."""
    cpeak = compute_peak(name, D, bf16)
    t_mem, t_cmp = nbytes / HBM_PEAK, flops / cpeak
    if t_mem >= t_cmp:
        achieved = nbytes / seconds / 1e9
        out = dict(kernel=name, bound='hbm', achieved=round(achieved, 2), peak=HBM_PEAK / 1e9, unit='GB/s',
                   frac=round(achieved / (HBM_PEAK / 1e9), 4), algorithmic_bytes=int(nbytes))
    else:
        achieved = flops / seconds / 1e12
        out = dict(kernel=name, bound='mfma', achieved=round(achieved, 3), peak=round(cpeak / 1e12, 1), unit='TFLOP/s',
                   frac=round(achieved / (cpeak / 1e12), 4), algorithmic_flops=int(flops))
    floors = {'hbm': t_mem, 'mfma': t_cmp}
    if valu is not None and valu[0]:
        t_valu = valu_floor(valu[0])
        floors['valu'] = t_valu
        out['valu'] = dict(insts_per_launch=int(valu[0]), floor_us=round(t_valu * 1e6, 2),
                           frac=round(t_valu / seconds, 4), source=valu[1],
                           model='4 cycles per wave64 VALU instruction on 1,024 SIMDs at 2.4 GHz')
    out['floors_us'] = {k: round(v * 1e6, 2) for k, v in floors.items()}
    out['limiter'] = max(floors, key=floors.get)
    return out
