"""Algorithmic FLOPs and HBM bytes per launch of a TriModalPlan step.

"Algorithmic" = the minimum the math needs: every input read once, every output written once,
no recomputation (the attention backward's recomputed S / dP are not counted).  fp32 (4 B).
Per attention-block instance (batch row b, block j), with n_kv = 1 (k is v):
  fwd flops = 4*Tq*Tk*D;  bytes = 4*(2*Tq*D + Tk*D) + 4*Tk + 8*H*Tq + 4*H*Tq*Tk*(r_in + r_out)
  bwd flops = 10*Tq*Tk*D; bytes = 4*(Tq*D*(q, x, dx, dq r+w) + Tk*D*(kv, dkv)) + 4*Tk + 8*H*Tq
          (+ S_prev, ds_next reads, ds_prev write when chained)
Peaks (MI355X_MICROARCH.md): HBM 8.0 TB/s; fp32 MFMA (= vector rate) 157.3 TFLOP/s; bf16 MFMA
2.5 PFLOP/s dense.  Kernels whose fp32 products run as bf16 parts (split.h) are priced against the
bf16 peak divided by the bf16 products per fp32 product: the block epilogues and the weight
gradients (six products) at 2.5 P / 6 = 417 TFLOP/s of fp32 work.  The attention kernels mix fp32
MFMA (forward P.V) and split products and are priced at the fp32 MFMA peak (they are HBM-bound at
every benched shape).  bf16 path (MEP_PREC_BF16): one bf16 product per product, every matrix
kernel priced at the bf16 peak; the bytes are the same (fp32 storage).
"""
from .trimodal import MODS

HBM_PEAK = 8.0e12
F32_PEAK = 157.3e12
BF16_PEAK = 2.5e15
COMPUTE_PEAK = {'mep_block_epi_fwd': BF16_PEAK / 6, 'mep_block_epi_bwd': BF16_PEAK / 6, 'mep_wgrad': BF16_PEAK / 6}


def launch_costs(plan):
    """{launch name: (flops, bytes)} for one eager training step of the plan (summed over the
    layers when a launch repeats)."""
    if not hasattr(plan, 'ntok') or not hasattr(plan, 'Xcat'):
        return rf_launch_costs(plan)
    sp, B = plan.spec, plan.B
    D, H = sp.D, sp.H
    out = {}

    def add(name, f, b):
        f0, b0 = out.get(name, (0, 0))
        out[name] = (f0 + f, b0 + b)

    for e in range(2):
        for m, d in zip(MODS, sp.dims):
            n = plan.ntok[m]
            add('mep_unify', 2 * n * D * d, 4 * (n * d + n * D + D * d))
    for blk in plan.blocks:
        Tq, Tk = blk['Tq'], blk['Tk']
        r_in = 1 if blk['i'] > 0 else 0
        r_out = 1 if 'S' in blk else 0
        s_bytes = 4 * H * Tq * Tk
        add('mep_attn_fwd', B * 4 * Tq * Tk * D,
            B * (4 * (2 * Tq * D + Tk * D) + 4 * Tk + 8 * H * Tq + s_bytes * (r_in + r_out)))
        n = B * Tq
        add('mep_block_epi_fwd', 2 * n * D * 3 * D + 8 * n * D, 4 * n * D * 5 + 8 * n + 4 * 3 * D * D + 8 * D)
        # upstream gradient formed from this block's dpooled / argmax slices (B x 3D), not read
        # as [n, D] rows (the pool backward is folded into this launch)
        add('mep_block_epi_bwd', 2 * n * D * 3 * D + 10 * n * D,
            4 * n * D * 6 + 8 * n + 4 * 3 * D * D + 4 * (n // 64 + 1) * 2 * D + 4 * B * 3 * D)
        chained = s_bytes * ((1 if r_out else 0) + (1 if r_in else 0) * 2)
        add('mep_attn_bwd', B * 10 * Tq * Tk * D,
            B * (4 * (5 * Tq * D + 2 * Tk * D) + 4 * Tk + 8 * H * Tq + chained))
        add('mep_wgrad', 2 * n * D * 3 * D, 4 * n * D * 5)
    for e in range(2):
        for m, d in zip(MODS, sp.dims):
            n = plan.ntok[m]
            add('mep_wgrad', 2 * n * D * d, 4 * n * (D + d))
    for e in range(2):
        add('mep_pool_fwd', B * plan.Ttot * plan.C, 4 * B * (plan.Ttot * plan.C + 2 * plan.C) + 4 * B * plan.C)
    return out


def rf_launch_costs(plan):
    """Attention launches of a realformer plan (RealformerPlan): K and V separately projected
    (n_kv = 2), the residual scores carried between the chain's layers."""
    sp, R = plan.spec, plan.R
    D, H = sp.D, sp.H
    out = {}

    def add(name, f, b):
        f0, b0 = out.get(name, (0, 0))
        out[name] = (f0 + f, b0 + b)
    for blk in plan.blocks:
        Tq, Tk = blk['Tq'], blk['Tk']
        r_in = 1 if blk['i'] > 0 else 0
        r_out = 1 if 'S' in blk else 0
        s_bytes = 4 * H * Tq * Tk
        add('mep_attn_fwd', R * 4 * Tq * Tk * D,
            R * (4 * (2 * Tq * D + 2 * Tk * D) + 4 * Tk + 8 * H * Tq + s_bytes * (r_in + r_out)))
        chained = s_bytes * ((1 if r_out else 0) + (1 if r_in else 0) * 2)
        add('mep_attn_bwd', R * 10 * Tq * Tk * D,
            R * (4 * (5 * Tq * D + 4 * Tk * D) + 4 * Tk + 8 * H * Tq + chained))
    return out


def roofline_entry(name, flops, nbytes, seconds, bf16=False):
    """The bench's roofline object for one kernel: bound = the larger of the two ideal times."""
    cpeak = BF16_PEAK if bf16 else COMPUTE_PEAK.get(name, F32_PEAK)
    t_mem, t_cmp = nbytes / HBM_PEAK, flops / cpeak
    if t_mem >= t_cmp:
        achieved = nbytes / seconds / 1e9
        return dict(kernel=name, bound='hbm', achieved=round(achieved, 2), peak=HBM_PEAK / 1e9, unit='GB/s',
                    frac=round(achieved / (HBM_PEAK / 1e9), 4), algorithmic_bytes=int(nbytes))
    achieved = flops / seconds / 1e12
    return dict(kernel=name, bound='mfma', achieved=round(achieved, 3), peak=round(cpeak / 1e12, 1), unit='TFLOP/s',
                frac=round(achieved / (cpeak / 1e12), 4), algorithmic_flops=int(flops))
