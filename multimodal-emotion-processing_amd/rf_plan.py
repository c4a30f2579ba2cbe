"""Execution plan of the others/realformer.py family on libmep_hip: ``Multi_class`` encoders under
the ``State_Transfer`` head, and the single-chain "text encoder" of BASELINE cfg2.

The P utterances of a State_Transfer batch share the encoder weights and are independent until
the gate recurrence (realformer.py:272-286), so the plan encodes all R = B*P utterances as ONE
batch (one grouped launch per stage instead of P Python iterations), and only the tiny
sigmoid/tanh recurrence runs per batch row (mep_rf_head).

Step anatomy
  forward   unify GEMM (+ position-embedding table) -> [w_qkv.1; w_qkv.2] KV projections of every
            block and the layer-0 Q projections (one grouped GEMM) -> per layer: Q projections
            (layers > 0), attention core (K != V), RealFormer epilogue (proj, a-residual LN1,
            FFN, b-residual LN2) -> mean+max pool -> fully_connected GEMM -> fused head
            (LN, ReLU, classifier, gate recurrence, circle loss, and its backward)
  backward  dpooled GEMM, pool backward, per layer (reverse): epilogue backward, attention
            backward, dQ / dKV input-gradient GEMMs; per-modality gradient sums; every weight
            gradient in one split-K launch; column sums for biases, LayerNorms, a/b/c, position
            tables and the head.
HBM layout: K and V projections of a block share one [ntok, 2D] buffer (one GEMM against the
adjacent [w_qkv.1; w_qkv.2] weights, one [ntok, 2D] gradient); last-layer outputs are written
straight into the pooled tensor [R, T_l+T_a+T_v, 3D] (torch.cat at realformer.py:258-261).
"""
import ctypes

import torch

from . import _lib
from ._lib import (AttnBwdDesc, AttnDesc, ColsumDesc, DescArray, GemmDesc, PoolDesc, RfEpiBwdDesc, RfEpiDesc,
                   RfHeadDesc, Rows, SumDesc, launch)
from .trimodal import (CHAINS, MODS, TIME_ORDER, UNIFY_NAMES, _norm_args, cdiv, crows, make_wgrad, reduce_blocks,
                       reduce_map, reduce_mapped, rows)

RF_SPLITQ = _lib.switch('MEP_RF_SPLITQ', '1') != '0'   # attention backward: query tiles over 4 waves
# unify + projections of each modality in one launch (mep_rfw_front) up to RF_FRONT_MAX_TILES
# 16-token tiles per step (cfg2's chain, 200: 27.5 -> 19.7 us); larger plans keep the GEMM
# launches (State_Transfer, 3600 tiles: 196 us on mep_wgemm_ws against 373 us on the front kernel,
# whose per-tile weight streaming from L2 grows with the tile count); 0: never
RF_FRONT = _lib.switch('MEP_RF_FRONT', '1') != '0'
RF_FRONT_MAX_TILES = 1024
# the input-gradient GEMMs and their per-modality sums in one launch (mep_wgemm_sum) when every
# sum has at most 4 sources, each the output of one of those GEMMs (cfg2's chain); 0: never
RF_WGEMM_SUM = _lib.switch('MEP_RF_WGEMM_SUM', '1') != '0'

NC = 6  # State_Transfer classes (realformer.py:268-269)
POS_NAMES = {'l': 'linguistic_position', 'v': 'visual_position', 'a': 'acoustic_position'}


class RealformerSpec:
    """Static description of a Multi_class encoder (+ optional State_Transfer head).

    prefix: state_dict prefix of the Multi_class ('feature.' under State_Transfer).
    chains: the (query, key) modality chains to run (all 9 for Multi_class; [('l', 'l')] for the
    cfg2 text chain, whose output is the last block's output instead of the pooled head)."""

    def __init__(self, D, H, n_layers, FD, dims, T, prefix='feature.', chains=CHAINS, head=True):
        assert D == 16 * H and D % 32 == 0 and D <= 128, 'kernels need hd = 16 and D in {32,64,96,128}'
        assert FD in (D, 2 * D), 'mep_rf_epi is compiled for FFN in {1, 2}'
        self.D, self.H, self.nl, self.FD = D, H, n_layers, FD
        self.dims = dict(zip(MODS, dims))
        self.Tlen = dict(zip(MODS, T))
        self.prefix = prefix
        self.chains = tuple(chains)
        self.head = head
        self.mods = tuple(m for m in MODS if any(m in c for c in self.chains))
        assert not head or len(self.chains) == 9

    def block_name(self, j, i):
        """chain j, layer i -> multimodal_blocks index (realformer.py:232-256)"""
        return self.prefix + 'multimodal_blocks.%d.' % (self.nl * CHAINS.index(self.chains[j]) + i)

    def no_grad_params(self, all_names):
        """Parameters that never receive a gradient: c of every chain's first layer (its scores
        input is None, realformer.py:187-190) and everything outside the chains / head run."""
        used = set()
        for m in self.mods:
            used.add(self.prefix + 'unify_dimension.%s.weight' % UNIFY_NAMES[m])
            used.add(self.prefix + '%s.position_embeddings.weight' % POS_NAMES[m])
        blocks = [self.block_name(j, i) for j in range(len(self.chains)) for i in range(self.nl)]
        heads = [self.prefix + 'fully_connected.', self.prefix + 'normalization.', 'classifier.', 'trans']
        out = []
        for n in all_names:
            if n in used:
                continue
            blk = [b for b in blocks if n.startswith(b)]
            if blk:
                first = int(blk[0].split('.')[-2]) % self.nl == 0
                if n == blk[0] + 'c' and first:
                    out.append(n)
                continue
            if self.head and any(n.startswith(h) for h in heads):
                continue
            out.append(n)
        return out


class RealformerPlan:
    def __init__(self, spec, flat, B, P, device):
        self.spec, self.flat = spec, flat
        self.B, self.P = B, P
        self.R = R = B * P
        self.device = dev = torch.device(device)
        sp = spec
        D, H, nl, FD = sp.D, sp.H, sp.nl, sp.FD
        # wave-tiled kernels on pre-split weights (csrc/rfw.hip: mep_wsplit, mep_wgemm,
        # mep_rfw_epi_*); MEP_RFW=0 keeps the LDS-tiled f32-MFMA kernels (A/B runs)
        self.rfw = _lib.RFW
        f32 = dict(dtype=torch.float32, device=dev)
        self.T = {m: sp.Tlen[m] for m in sp.mods}
        self.ntok = {m: R * self.T[m] for m in sp.mods}
        assert max(self.ntok.values()) < 1 << 22, 'row views are limited to 2^22 rows (csrc/common.h row_off)'
        # ---------------- static inputs ([R, T, d] = the reference's [B, P, T, d])
        # feature rows padded to a multiple of 4 floats (zeros, never written): the token GEMMs
        # read them in 16-byte blocks (MEP_WGEMM_XVEC); x_in[m] is the [R, T, d] view
        self.x_pad = {m: torch.zeros(R, self.T[m], -(-sp.dims[m] // 4) * 4, **f32) for m in sp.mods}
        self.x_in = {m: self.x_pad[m][..., :sp.dims[m]] for m in sp.mods}
        self.x_padded = frozenset(t.data_ptr() for t in self.x_pad.values())
        self.m_in = {m: torch.zeros(R, self.T[m], **f32) for m in sp.mods}
        self.U = {m: torch.zeros(self.ntok[m], D, **f32) for m in sp.mods}
        self.dU = {m: torch.zeros(self.ntok[m], D, **f32) for m in sp.mods}
        self.loss = torch.zeros(1, **f32)
        if sp.head:
            self.labels = torch.zeros(B, P, NC, dtype=torch.int64, device=dev)
            self.umask = torch.zeros(B, P, dtype=torch.int64, device=dev)
            self.Ttot = sum(self.T.values())
            self.C = 3 * D
            self.Xcat = torch.zeros(R, self.Ttot, self.C, **f32)
            self.dXcat = torch.zeros_like(self.Xcat)
            self.pooled = torch.zeros(R, 2 * self.C, **f32)
            self.dpooled = torch.zeros_like(self.pooled)
            self.argmax = torch.zeros(R, self.C, dtype=torch.int32, device=dev)
            self.fc = torch.zeros(R, D, **f32)
            self.h = torch.zeros(R, D, **f32)
            self.dfc = torch.zeros(R, D, **f32)
            self.d12 = torch.zeros(R, 2 * NC, **f32)
            self.out = torch.zeros(B, P, NC, **f32)
            self.row_loss = torch.zeros(B, **f32)
            self.head_partial = torch.zeros(B, 2 * D + NC * NC, **f32)
            self.toff, t = {}, 0
            for m in TIME_ORDER:
                self.toff[m] = t
                t += self.T[m]
        self.blocks = []
        for j, (qm, km) in enumerate(sp.chains):
            for i in range(nl):
                self.blocks.append(self._make_block(j, i, qm, km))
        nq_all = sum(b['nq'] for b in self.blocks)
        self.dQP_all = torch.zeros(nq_all, D, **f32)   # attention dq accumulates: zeroed per step
        off = 0
        for b in self.blocks:
            b['dQP'] = self.dQP_all[off:off + b['nq']]
            off += b['nq']
        if not sp.head:
            last = self._blk(0, nl - 1)
            self.out_chain = last['OUT']
            self.dout_chain = torch.zeros_like(last['OUT'])
        self._build()

    # ------------------------------------------------------------------ buffers
    def _make_block(self, j, i, qm, km):
        sp, R = self.spec, self.R
        D, H, FD, nl = sp.D, sp.H, sp.FD, sp.nl
        f32 = dict(dtype=torch.float32, device=self.device)
        Tq, Tk = self.T[qm], self.T[km]
        nq, nk = R * Tq, R * Tk
        blk = dict(idx=len(self.blocks), j=j, i=i, qm=qm, km=km, Tq=Tq, Tk=Tk, nq=nq, nk=nk,
                   pre=sp.block_name(j, i))
        for name in ('QP', 'X', 'XP', 'H', 'F', 'dXP', 'dX', 'dF', 'dQin'):
            blk[name] = torch.zeros(nq, D, **f32)
        blk['F1'] = torch.zeros(nq, FD, **f32)
        blk['dF1'] = torch.zeros(nq, FD, **f32)
        blk['KV'] = torch.zeros(nk, 2 * D, **f32)
        blk['dKV2'] = torch.zeros(nk, 2 * D, **f32)
        blk['dKVin'] = torch.zeros(nk, D, **f32)
        blk['estat'] = torch.zeros(nq, 4, **f32)
        blk['astat'] = torch.zeros(3 * R * H * Tq, **f32)   # (max, 1/sum) per row, then the residual rows' S_prev means
        blk['partial'] = torch.zeros(cdiv(nq, _lib.rf_bwd_rows(self.rfw)), _lib.rf_partial_stride(D, FD), **f32)
        if i < nl - 1 or not sp.head:
            blk['OUT'] = torch.zeros(nq, D, **f32)
        if i < nl - 1:
            blk['S'] = torch.zeros(R, H, Tq, Tk, **f32)
        if i >= 1:
            blk['dSprev'] = torch.zeros(R, H, Tq, Tk, **f32)
            blk['dc_partial'] = torch.zeros(_lib.attn_dc_slots(R, H, Tk), **f32)
        blk['col'] = (CHAINS.index(sp.chains[j]) % 3) * D
        return blk

    def _blk(self, j, i):
        return self.blocks[j * self.spec.nl + i]

    def _q_rows(self, blk):
        if blk['i'] == 0:
            return crows(self.U[blk['qm']], blk['Tq'], self.spec.D)
        return self._out_rows(self._blk(blk['j'], blk['i'] - 1))

    def _out_rows(self, blk):
        D = self.spec.D
        if 'OUT' in blk:
            return crows(blk['OUT'], blk['Tq'], D)
        return rows(self.Xcat, blk['Tq'], self.Ttot * self.C, self.C, self.toff[blk['qm']] * self.C + blk['col'])

    def _dout_rows(self, blk):
        D, sp = self.spec.D, self.spec
        if blk['i'] < sp.nl - 1:
            return crows(self._blk(blk['j'], blk['i'] + 1)['dQin'], blk['Tq'], D)
        if not sp.head:
            return crows(self.dout_chain, blk['Tq'], D)
        return rows(self.dXcat, blk['Tq'], self.Ttot * self.C, self.C, self.toff[blk['qm']] * self.C + blk['col'])

    def _in_rows(self, m):
        T, dp = self.T[m], self.x_pad[m].shape[-1]
        return rows(self.x_pad[m], T, T * dp, dp)

    def _kv_rows(self, blk, which, t):
        """K (which=0) or V (which=1) half of a [ntok, 2D] buffer t"""
        D = self.spec.D
        return rows(t, blk['Tk'], blk['Tk'] * 2 * D, 2 * D, which * D)

    # ------------------------------------------------------------------ descriptors
    def _build_front(self, ud, pd, dev):
        """mep_rfw_front launches (unify + the projections of its output in one kernel per
        modality) when every modality's launch fits the kernel's contract; else self.front = None
        and the forward runs the unify and projection GEMM launches"""
        self.front = None
        if not RF_FRONT or self.spec.D != 96 or sum(cdiv(d.ntok, 16) for d in ud) > RF_FRONT_MAX_TILES:
            return
        groups = {}
        for dsc in ud:
            m = next(k for k in self.spec.mods if dsc.y.ptr == self.U[k].data_ptr())
            outs = [q for q in pd if q.x.ptr == self.U[m].data_ptr()]
            npk = -(-dsc.K // 32)
            tiles = sum(q.N // 16 for q in outs)
            ok = (npk in (2, 3, 10) and dsc.N == 96 and not dsc.relu and not dsc.accumulate and
                  dsc.x.ptr in self.x_padded and 0 < len(outs) <= _lib.RF_FRONT_MAX_OUT and
                  6 <= tiles <= _lib.RF_FRONT_MAX_TILES and
                  all(q.K == 96 and q.N % 16 == 0 and q.alpha == 1.0 and not (q.bias or q.table or q.accumulate or q.relu)
                      for q in outs) and
                  # the kernel reads U from its LDS exchange at the unify's token index and stores
                  # each output row with 16-byte stores: the projections read U's dense rows of the
                  # same tokens and write aligned rows
                  all(q.ntok == dsc.ntok and (q.x.sB, q.x.sT, q.x.T) == (dsc.y.sB, dsc.y.sT, dsc.y.T) and
                      dsc.y.sT == 96 and q.y.ptr % 16 == 0 and q.y.sB % 4 == 0 and q.y.sT % 4 == 0
                      for q in outs))
            if not ok:
                return
            fd = _lib.RfFrontDesc(unify=dsc, n_out=len(outs), n_tiles=tiles)
            t = 0
            for o, q in enumerate(outs):
                fd.out[o] = _lib.RfFrontOut(w=q.w, y=q.y, N=q.N)
                for lt in range(q.N // 16):
                    fd.tile_map[t] = (o << 8) | lt
                    t += 1
            groups.setdefault(npk, []).append((fd, dsc.ntok))
        self.front = [(DescArray(_lib.RfFrontDesc, [fd for fd, _ in g], dev), cdiv(max(n for _, n in g), 16), npk)
                      for npk, g in sorted(groups.items())]

    def _attn_desc(self, blk):
        sp, fl, D = self.spec, self.flat, self.spec.D
        prev = self._blk(blk['j'], blk['i'] - 1) if blk['i'] > 0 else None
        return AttnDesc(q=crows(blk['QP'], blk['Tq'], D), k=self._kv_rows(blk, 0, blk['KV']),
                        v=self._kv_rows(blk, 1, blk['KV']), x=crows(blk['X'], blk['Tq'], D),
                        mask=self.m_in[blk['km']].data_ptr(), mask_sB=blk['Tk'],
                        s_prev=prev['S'].data_ptr() if prev is not None else 0, c=fl.ptr(blk['pre'] + 'c'),
                        s_out=blk['S'].data_ptr() if 'S' in blk else 0, stats=blk['astat'].data_ptr(),
                        B=self.R, H=sp.H, Tq=blk['Tq'], Tk=blk['Tk'])

    def _epi_desc(self, blk):
        sp, fl, D, Tq = self.spec, self.flat, self.spec.D, blk['Tq']
        p = blk['pre']
        return RfEpiDesc(q=self._q_rows(blk), x=crows(blk['X'], Tq, D), xp=crows(blk['XP'], Tq, D),
                         h=crows(blk['H'], Tq, D), f1=crows(blk['F1'], Tq, sp.FD), f=crows(blk['F'], Tq, D),
                         out=self._out_rows(blk), wp=fl.ptr(p + 'proj.weight'), w1=fl.ptr(p + 'ffn.0.weight'),
                         b1=fl.ptr(p + 'ffn.0.bias'), w2=fl.ptr(p + 'ffn.2.weight'), b2=fl.ptr(p + 'ffn.2.bias'),
                         ln1_w=fl.ptr(p + 'norm1.weight'), ln1_b=fl.ptr(p + 'norm1.bias'),
                         ln2_w=fl.ptr(p + 'norm2.weight'), ln2_b=fl.ptr(p + 'norm2.bias'),
                         a=fl.ptr(p + 'a'), b=fl.ptr(p + 'b'), stats=blk['estat'].data_ptr(),
                         ntok=blk['nq'], D=D, FD=sp.FD, wparts=blk.get('wparts', 0),
                         wq_next=blk.get('wq_next', 0), qp_next=blk.get('qp_next', Rows()),
                         zero=crows(blk['dQP'], Tq, D) if self.rfw else Rows())

    def _epi_bwd_desc(self, blk):
        D, Tq, FD = self.spec.D, blk['Tq'], self.spec.FD
        return RfEpiBwdDesc(f=self._epi_desc(blk), dout=self._dout_rows(blk), dout2=Rows(),
                            df=crows(blk['dF'], Tq, D), df1=crows(blk['dF1'], Tq, FD),
                            dxp=crows(blk['dXP'], Tq, D), dx=crows(blk['dX'], Tq, D),
                            dq=crows(blk['dQin'], Tq, D), partial=blk['partial'].data_ptr(), dq_accumulate=0,
                            wq_in=blk.get('wq_in', 0), dqp_in=blk.get('dqp_in', Rows()))

    def _attn_bwd_desc(self, blk):
        D = self.spec.D
        nxt = self._blk(blk['j'], blk['i'] + 1) if blk['i'] < self.spec.nl - 1 else None
        return AttnBwdDesc(f=self._attn_desc(blk), dx=crows(blk['dX'], blk['Tq'], D),
                           dq=crows(blk['dQP'], blk['Tq'], D), dk=self._kv_rows(blk, 0, blk['dKV2']),
                           dv=self._kv_rows(blk, 1, blk['dKV2']),
                           ds_next=nxt['dSprev'].data_ptr() if nxt is not None else 0,
                           ds_prev=blk['dSprev'].data_ptr() if 'dSprev' in blk else 0,
                           dc_partial=blk['dc_partial'].data_ptr() if 'dc_partial' in blk else 0)

    def _wkv(self, blk):
        """[w_qkv.1; w_qkv.2] as one [2D, D] matrix (adjacent in the flat buffer)"""
        fl, D, p = self.flat, self.spec.D, blk['pre']
        k, v = fl.offsets[p + 'w_qkv.1.weight'], fl.offsets[p + 'w_qkv.2.weight']
        assert v == k + D * D, 'w_qkv.1 / w_qkv.2 must be adjacent in the flat buffer'
        return p + 'w_qkv.1.weight'

    def _build(self):
        sp, fl, R, D, H, nl, FD = self.spec, self.flat, self.R, self.spec.D, self.spec.H, self.spec.nl, self.spec.FD
        dev = self.device
        g = fl.gptr
        gemm = dict(bias=0, table=0, accumulate=0, relu=0, alpha=1.0)
        # unify: Conv1d k=1 (== Linear on the feature axis) + position embedding table
        ud = []
        for m in sp.mods:
            d, T = sp.dims[m], self.T[m]
            ud.append(GemmDesc(x=self._in_rows(m), y=crows(self.U[m], T, D),
                               w=fl.ptr(sp.prefix + 'unify_dimension.%s.weight' % UNIFY_NAMES[m]),
                               bias=0, table=fl.ptr(sp.prefix + '%s.position_embeddings.weight' % POS_NAMES[m]),
                               ntok=self.ntok[m], N=D, K=d, ldw=d, w_nt=1, accumulate=0, relu=0, alpha=1.0))
        self.t_unify = max(cdiv(self.ntok[m], 64) for m in sp.mods)
        # projections: KV of every block + Q of layer 0 (all read U only)
        pd = []
        for blk in self.blocks:
            pd.append(GemmDesc(x=crows(self.U[blk['km']], blk['Tk'], D), y=crows(blk['KV'], blk['Tk'], 2 * D),
                               w=fl.ptr(self._wkv(blk)), ntok=blk['nk'], N=2 * D, K=D, ldw=D, w_nt=1, **gemm))
            if blk['i'] == 0:
                pd.append(GemmDesc(x=self._q_rows(blk), y=crows(blk['QP'], blk['Tq'], D),
                                   w=fl.ptr(blk['pre'] + 'w_qkv.0.weight'), ntok=blk['nq'], N=D, K=D, ldw=D,
                                   w_nt=1, **gemm))
        self.t_proj = max(cdiv(b['nk'], 64) for b in self.blocks)
        self.d_q, self.d_attn, self.d_epi, self.t_attn, self.t_epi = [], [], [], [], []
        self.t_epif, self.t_epib = [], []   # mep_rf_epi_fwd / _bwd workgroups (t_epi: 64-token tiles)
        self.d_epib, self.d_attnb, self.t_attnb, self.d_ingrad = [], [], [], []
        self.f_attn, self.f_attnb = [], []
        qd, igd = [], []
        for i in range(nl):
            layer = [b for b in self.blocks if b['i'] == i]
            qd.append([GemmDesc(x=self._q_rows(b), y=crows(b['QP'], b['Tq'], D), w=fl.ptr(b['pre'] + 'w_qkv.0.weight'),
                                ntok=b['nq'], N=D, K=D, ldw=D, w_nt=1, **gemm) for b in layer] if i > 0 else [])
            ad = [self._attn_desc(b) for b in layer]
            self.d_attn.append(DescArray(AttnDesc, ad, dev))
            geo = _lib.attn_geometry(ad)
            sq, sq_tiles = _lib.attn_fwd_splitq(ad) if RF_SPLITQ else (0, None)
            self.t_attn.append(sq_tiles or geo[0])
            self.t_attnb.append(geo[1])
            self.f_attn.append(geo[2] | sq)
            self.t_epi.append(max(cdiv(b['nq'], 16 if self.rfw else 64) for b in layer))
            ab = [self._attn_bwd_desc(b) for b in layer]
            self.d_attnb.append(DescArray(AttnBwdDesc, ab, dev))
            self.f_attnb.append(_lib.attn_bwd_flags(ab) | (_lib.attn_bwd_splitq(ab) if RF_SPLITQ else 0))
            ig = []
            for b in layer:
                # dq_in += dQP W_q  (onto the residual dz1 the epilogue backward wrote)
                ig.append(GemmDesc(x=crows(b['dQP'], b['Tq'], D), y=crows(b['dQin'], b['Tq'], D),
                                   w=fl.ptr(b['pre'] + 'w_qkv.0.weight'), bias=0, table=0, ntok=b['nq'], N=D, K=D,
                                   ldw=D, w_nt=0, accumulate=1, relu=0, alpha=1.0))
                # dkv_in = [dK | dV] [W_k; W_v]
                ig.append(GemmDesc(x=crows(b['dKV2'], b['Tk'], 2 * D), y=crows(b['dKVin'], b['Tk'], D),
                                   w=fl.ptr(self._wkv(b)), ntok=b['nk'], N=D, K=2 * D, ldw=D, w_nt=0, **gemm))
            igd.append(ig)
        self.t_ingrad = max(max(cdiv(b['nq'], 64), cdiv(b['nk'], 64)) for b in self.blocks)
        ig_all = []
        if self.rfw:
            # layer i's epilogue forward also runs layer i+1's query projection and layer i's
            # epilogue backward adds layer i+1's dQP W_q to its upstream gradient, so the q GEMMs
            # of layers > 0 go away and the remaining input-gradient GEMMs (layer-0 dq_in, every
            # dkv_in: they only feed the per-modality sums) run as one launch after the backward
            qd = [[] for _ in range(nl)]
            ig_all = [x for l_, ig in enumerate(igd) for x in ig if l_ == 0 or x.K == 2 * D]
            igd = [[] for _ in range(nl)]
            # every token GEMM and epilogue Linear on mep_wsplit parts (refreshed at the start of
            # each forward): W' = the weight as it is (w_nt) or its transpose (dY W products)
            arena = _lib.PartsArena()
            patch = []
            for dsc in ud + pd + ig_all:
                patch.append((dsc, arena.add(dsc.w, dsc.N, dsc.K, dsc.ldw, 0 if dsc.w_nt else 1)))
            fused = []
            for b in self.blocks:
                if b['i'] < nl - 1:
                    nxt = self._blk(b['j'], b['i'] + 1)
                    wq = fl.ptr(nxt['pre'] + 'w_qkv.0.weight')
                    fused.append((b, nxt, arena.add(wq, D, D, D, 0), arena.add(wq, D, D, D, 1)))
            epi_off = [arena.add_epi(D, FD, fl.ptr(b['pre'] + 'proj.weight'), fl.ptr(b['pre'] + 'ffn.0.weight'),
                                     fl.ptr(b['pre'] + 'ffn.2.weight')) for b in self.blocks]
            self.wparts, self.d_wsplit, self.t_wsplit = arena.build(dev)
            for dsc, off in patch:
                dsc.w = self.wparts.data_ptr() + off
            for b, off in zip(self.blocks, epi_off):
                b['wparts'] = self.wparts.data_ptr() + off
            self._build_front(ud, pd, dev)
            for b, nxt, o_fwd, o_bwd in fused:
                b['wq_next'] = self.wparts.data_ptr() + o_fwd
                b['qp_next'] = crows(nxt['QP'], nxt['Tq'], D)
                b['wq_in'] = self.wparts.data_ptr() + o_bwd
                b['dqp_in'] = crows(nxt['dQP'], nxt['Tq'], D)
            self.t_unify = max(cdiv(self.ntok[m], 16) for m in sp.mods)
            self.t_proj = max(cdiv(b['nk'], 16) for b in self.blocks)
            self.t_ingrad = max(max(cdiv(b['nq'], 16), cdiv(b['nk'], 16)) for b in self.blocks)
        self.d_unify = DescArray(GemmDesc, ud, dev)
        self.d_proj = DescArray(GemmDesc, pd, dev)
        self.d_q = [DescArray(GemmDesc, x, dev) for x in qd]
        self.d_ingrad = [DescArray(GemmDesc, x, dev) for x in igd]
        self.d_ingrad_all = DescArray(GemmDesc, ig_all, dev)
        for i in range(nl):
            layer = [b for b in self.blocks if b['i'] == i]
            self.d_epi.append(DescArray(RfEpiDesc, [self._epi_desc(b) for b in layer], dev))
            self.t_epif.append(max(cdiv(b['nq'], _lib.rf_epi_rows(self.spec.D, self.rfw)) for b in layer))
            self.t_epib.append(max(cdiv(b['nq'], _lib.rf_bwd_rows(self.rfw)) for b in layer))
            self.d_epib.append(DescArray(RfEpiBwdDesc, [self._epi_bwd_desc(b) for b in layer], dev))
        # per-modality input-gradient sums
        sd = []
        for m in sp.mods:
            T = self.T[m]
            srcs = [crows(self._blk(j, 0)['dQin'], T, D) for j, (qm, km) in enumerate(sp.chains) if qm == m]
            srcs += [crows(self._blk(j, i)['dKVin'], T, D) for j, (qm, km) in enumerate(sp.chains) if km == m
                     for i in range(nl)]
            assert len(srcs) <= _lib.SUM_MAX_SRC
            sd.append(SumDesc(src=(Rows * _lib.SUM_MAX_SRC)(*srcs), out=crows(self.dU[m], T, D), n_src=len(srcs),
                              ntok=self.ntok[m], D=D, accumulate=0))
        self.d_sum = DescArray(SumDesc, sd, dev)
        self.t_sum = min(1024, max(cdiv(self.ntok[m] * D // 4, 256) for m in sp.mods))
        self.d_isum = self._fuse_sums(ig_all, sd, dev) if self.rfw and RF_WGEMM_SUM and ig_all else None
        if sp.head:
            self._build_head()
        self._build_grads()

    def _fuse_sums(self, ig_all, sd, dev):
        """mep_wgemm_sum descriptors replacing the ingrad launch + mep_sum_rows, or None when some
        sum has more than WGEMM_SUM_MAX sources, a source no single GEMM writes, or a GEMM feeds
        no sum (or the ingrad launch would take the weight-stationary kernel)"""
        if self.gemm_launcher(self.d_ingrad_all) != 'mep_wgemm':
            return None
        by_y = {}
        for g in ig_all:
            by_y.setdefault((g.y.ptr, g.y.sB, g.y.sT), []).append(g)
        out, used = [], 0
        for s in sd:
            if s.n_src > _lib.WGEMM_SUM_MAX or s.accumulate:
                return None
            src = []
            for k in range(s.n_src):
                r = s.src[k]
                g = by_y.get((r.ptr, r.sB, r.sT), [])
                if len(g) != 1 or g[0].ntok != s.ntok or g[0].N != s.D:
                    return None
                src.append(g[0])
            used += len(src)
            out.append(_lib.GemmSumDesc(src=(GemmDesc * _lib.WGEMM_SUM_MAX)(*src), n_src=len(src), out=s.out))
        if used != len(ig_all):
            return None
        return DescArray(_lib.GemmSumDesc, out, dev)

    def _build_head(self):
        sp, fl, R, D = self.spec, self.flat, self.R, self.spec.D
        dev = self.device
        pre = sp.prefix
        self.d_pool = DescArray(PoolDesc, [PoolDesc(x=self.Xcat.data_ptr(), dx=self.dXcat.data_ptr(),
                                                    pooled=self.pooled.data_ptr(), dpooled=self.dpooled.data_ptr(),
                                                    argmax=self.argmax.data_ptr(), B=R, T=self.Ttot, C=self.C)], dev)
        self.t_pool = R * cdiv(self.C, 32)
        self.t_poolb = R * cdiv(self.Ttot, 16)
        F = 2 * self.C
        self.d_fc = DescArray(GemmDesc, [GemmDesc(
            x=crows(self.pooled, 1, F), y=crows(self.fc, 1, D), w=fl.ptr(pre + 'fully_connected.weight'),
            bias=fl.ptr(pre + 'fully_connected.bias'), table=0, ntok=R, N=D, K=F, ldw=F, w_nt=1, accumulate=0,
            relu=0, alpha=1.0)], dev)
        self.d_fcb = DescArray(GemmDesc, [GemmDesc(
            x=crows(self.dfc, 1, D), y=crows(self.dpooled, 1, F), w=fl.ptr(pre + 'fully_connected.weight'),
            bias=0, table=0, ntok=R, N=F, K=D, ldw=F, w_nt=0, accumulate=0, relu=0, alpha=1.0)], dev)
        self.t_fc = cdiv(R, 64)
        # loss scale read by the head kernel at run time (mep_rf_head_desc.scale): one captured
        # graph serves every data-parallel share size
        self.head_scale = torch.full((1,), 1.0 / R, dtype=torch.float32, device=dev)
        self._head_scale = 1.0 / R
        self.head = RfHeadDesc(fc=self.fc.data_ptr(), ln_w=fl.ptr(pre + 'normalization.weight'),
                               ln_b=fl.ptr(pre + 'normalization.bias'), wc=fl.ptr('classifier.weight'),
                               bc=fl.ptr('classifier.bias'), trans=fl.ptr('trans'), labels=self.labels.data_ptr(),
                               umask=self.umask.data_ptr(), out=self.out.data_ptr(), h=self.h.data_ptr(),
                               d12=self.d12.data_ptr(), dfc=self.dfc.data_ptr(), row_loss=self.row_loss.data_ptr(),
                               partial=self.head_partial.data_ptr(), ext_dout=0, B=self.B, P=self.P, D=D,
                               compute_grad=1, loss_scale=1.0 / R, scale=self.head_scale.data_ptr())

    def _build_grads(self):
        sp, fl, R, D, FD = self.spec, self.flat, self.R, self.spec.D, self.spec.FD
        dev = self.device
        g = fl.gptr
        items = []
        for b in self.blocks:
            Tq, Tk, nq, nk, p = b['Tq'], b['Tk'], b['nq'], b['nk'], b['pre']
            items.append((crows(b['dQP'], Tq, D), D, nq, [(self._q_rows(b), D, g(p + 'w_qkv.0.weight'), D)]))
            items.append((crows(self.U[b['km']], Tk, D), D, nk,
                          [(crows(b['dKV2'], Tk, 2 * D), 2 * D, g(self._wkv(b)), D)], 1))
            items.append((crows(b['dXP'], Tq, D), D, nq, [(crows(b['X'], Tq, D), D, g(p + 'proj.weight'), D)]))
            items.append((crows(b['H'], Tq, D), D, nq, [(crows(b['dF1'], Tq, FD), FD, g(p + 'ffn.0.weight'), D)], 1))
            items.append((crows(b['dF'], Tq, D), D, nq, [(crows(b['F1'], Tq, FD), FD, g(p + 'ffn.2.weight'), FD)]))
        for m in sp.mods:
            d = sp.dims[m]
            items.append((crows(self.dU[m], self.T[m], D), D, self.ntok[m],
                          [(self._in_rows(m), d, g(sp.prefix + 'unify_dimension.%s.weight' % UNIFY_NAMES[m]), d)]))
        if sp.head:
            F = 2 * self.C
            items.append((crows(self.dfc, 1, D), D, R, [(crows(self.pooled, 1, F), F,
                                                         g(sp.prefix + 'fully_connected.weight'), F)]))
            items.append((crows(self.d12, 1, 2 * NC), 2 * NC, R, [(crows(self.h, 1, D), D, g('classifier.weight'), D)]))
        self.wg_partial, self.d_wgrad, self.t_wgrad, self.t_wgred = make_wgrad(items, dev)
        cs = []

        def col(partial, out, n_rows, n_cols, ld, not_grad=False):
            cs.append(ColsumDesc(partial=partial, out=out, n_rows=n_rows, n_cols=n_cols, ld=ld,
                                 accumulate=_lib.COLSUM_NOT_GRAD if not_grad else 0))

        S = _lib.rf_partial_stride(D, FD)
        for b in self.blocks:
            base, nt, p = b['partial'].data_ptr(), b['partial'].shape[0], b['pre']
            for k, (name, n) in enumerate((('norm2.weight', D), ('norm2.bias', D), ('norm1.weight', D),
                                           ('norm1.bias', D), ('ffn.2.bias', D))):
                col(base + 4 * k * D, g(p + name), nt, n, S)
            col(base + 4 * 5 * D, g(p + 'ffn.0.bias'), nt, FD, S)
            col(base + 4 * (5 * D + FD), g(p + 'a'), nt, 1, S)
            col(base + 4 * (5 * D + FD + 1), g(p + 'b'), nt, 1, S)
            if 'dc_partial' in b:
                col(b['dc_partial'].data_ptr(), g(p + 'c'), b['dc_partial'].numel(), 1, 1)
        for m in sp.mods:
            T = self.T[m]
            col(self.dU[m].data_ptr(), g(sp.prefix + '%s.position_embeddings.weight' % POS_NAMES[m]), R, T * D, T * D)
        if sp.head:
            pre = sp.prefix
            col(self.dfc.data_ptr(), g(pre + 'fully_connected.bias'), R, D, D)
            col(self.d12.data_ptr(), g('classifier.bias'), R, 2 * NC, 2 * NC)
            W = 2 * D + NC * NC
            hp = self.head_partial.data_ptr()
            col(hp, g(pre + 'normalization.weight'), self.B, D, W)
            col(hp + 4 * D, g(pre + 'normalization.bias'), self.B, D, W)
            col(hp + 8 * D, g('trans'), self.B, NC * NC, W)
            col(self.row_loss.data_ptr(), self.loss.data_ptr(), self.B, 1, 1, not_grad=True)   # the batch loss
        self.d_colsum = DescArray(ColsumDesc, cs, dev)
        self.t_colsum = max(cdiv(c.n_cols, 32) for c in cs)
        self.redmap = reduce_map(self.d_wgrad, self.d_colsum, None, dev)

    # ------------------------------------------------------------------ execution
    def set_global_rows(self, n):
        """Data-parallel share (mep_amd.dp): the masked circle-loss mean over B * P utterance slots
        (others/realformer.py:312) taken over the n global rows (None: the local B)."""
        rows = self.B if n is None else int(n)
        val = 1.0 / (rows * self.P)
        if val != self._head_scale:          # a device fill, no host sync
            self.head_scale.fill_(val)
            self._head_scale = val
        self.head.loss_scale = val
        return rows

    def set_row0(self, row0):
        pass                                 # no dropout on the realformer path

    def set_inputs(self, l, v, a, lm, vm, am, labels=None, umask=None):
        """Reference-shaped [B, P, T, d] features / [B, P, T] masks (or [B, T, d] / [B, T] for the
        single-utterance chain plan) into the resident buffers."""
        with torch.no_grad():
            for m, x, mk in (('l', l, lm), ('v', v, vm), ('a', a, am)):
                if m not in self.spec.mods:
                    continue
                self.x_in[m].copy_(x.reshape(self.x_in[m].shape))   # into the padded rows
                self.m_in[m].copy_(mk.reshape(self.m_in[m].shape))
            if labels is not None:
                self.labels.copy_(labels)
            if umask is not None:
                self.umask.copy_(umask)

    _drop = 0.0

    def set_dropout(self, p):
        if p != 0.0:
            raise NotImplementedError('mep_amd realformer path: DROP must be 0 (the reference value, '
                                      'others/realformer.py:37)')

    def advance_seed(self, stream=None):
        pass

    def forward(self, grad=True, rdrop=False, stream=None):
        sp, nl = self.spec, self.spec.nl
        assert not rdrop
        ex = (sp.D, sp.FD)
        if self.rfw:
            launch('mep_wsplit', self.d_wsplit, self.t_wsplit, stream)
        if getattr(self, 'front', None):
            for descs, tiles, npk in self.front:
                _lib.call('mep_rfw_front', descs.ptr, descs.n, tiles, npk, stream=stream)
        else:
            self._gemm(self.d_unify, self.t_unify, stream)
            self._gemm(self.d_proj, self.t_proj, stream)
        for i in range(nl):
            if i > 0:
                self._gemm(self.d_q[i], self.t_epi[i], stream)
            launch('mep_attn_fwd', self.d_attn[i], self.t_attn[i], stream, threads=self.f_attn[i])
            launch('mep_rfw_epi_fwd' if self.rfw else 'mep_rf_epi_fwd', self.d_epi[i], self.t_epif[i], stream, extra=ex)
        # rfw: the forward epilogues cleared the attention dq rows (mep_rf_epi_desc.zero); the
        # first backward after this forward may accumulate onto them
        self._dq_clean = self.rfw
        if sp.head:
            launch('mep_pool_fwd', self.d_pool, self.t_pool, stream)
            # the head's fully_connected (B x P rows, K = 2C = 576): on mep_tgemm's 128-row workgroups
            # it is 3 workgroups walking 18 K chunks (45 us at State_Transfer); mep_gemm spreads it
            _lib.gemm('mep_gemm', self.d_fc, self.t_fc, stream, tgemm=False)
            self.head.compute_grad = int(grad)
            self.head.ext_dout = 0
            _lib.call('mep_rf_head', ctypes.byref(self.head), stream=stream)

    def gemm_launcher(self, descs):
        """launch name a token-GEMM descriptor array runs under (bench.py / roofline.py)"""
        if not self.rfw:
            return _lib.gemm_launcher('mep_gemm', descs)
        return 'mep_wgemm_ws' if _lib.wgemm_ws_fits(descs.items) else 'mep_wgemm'

    def _gemm(self, descs, tiles, stream):
        """a token-GEMM launch: mep_wgemm on the arena's parts, or the mep_gemm path"""
        if self.rfw:
            if descs.n and self.gemm_launcher(descs) == 'mep_wgemm_ws':
                _lib.wgemm_ws(descs, stream, self.x_padded)
            elif descs.n:
                _lib.call('mep_wgemm', descs.ptr, descs.n, int(tiles), max(d.N for d in descs.items), stream=stream)
        else:
            _lib.gemm('mep_gemm', descs, tiles, stream)

    def backward(self, ext_dout=None, stream=None):
        """Backward from the fused loss (or from ext_dout: [B, P, 6] for the head, the last block's
        output gradient for the chain plan).  Writes every gradient into flat.grad."""
        sp, nl = self.spec, self.spec.nl
        ex = (sp.D, sp.FD)
        if sp.head:
            if ext_dout is not None:
                self.head.compute_grad = 1
                self.head.ext_dout = ext_dout.data_ptr()
                _lib.call('mep_rf_head', ctypes.byref(self.head), stream=stream)
                self.head.ext_dout = 0
            _lib.gemm('mep_gemm', self.d_fcb, self.t_fc, stream)
            launch('mep_pool_bwd', self.d_pool, self.t_poolb, stream)
        elif ext_dout is not None:
            self.dout_chain.copy_(ext_dout.reshape(self.dout_chain.shape))
        if not getattr(self, '_dq_clean', False):
            # the attention backward accumulates dq: a second backward of one forward (retain_graph)
            # or the round-2 kernels clear the rows here (rfw forwards clear them in their epilogues)
            self.dQP_all.zero_()
        self._dq_clean = False
        for i in reversed(range(nl)):
            launch('mep_rfw_epi_bwd' if self.rfw else 'mep_rf_epi_bwd', self.d_epib[i], self.t_epib[i], stream, extra=ex)
            launch('mep_attn_bwd', self.d_attnb[i], self.t_attnb[i], stream, threads=self.f_attnb[i])
            self._gemm(self.d_ingrad[i], self.t_ingrad, stream)
        if self.d_isum is not None:
            _lib.call('mep_wgemm_sum', self.d_isum.ptr, self.d_isum.n, int(self.t_ingrad), self.spec.D, stream=stream)
        else:
            self._gemm(self.d_ingrad_all, self.t_ingrad, stream)
            launch('mep_sum_rows', self.d_sum, self.t_sum, stream)
        launch('mep_wgrad', self.d_wgrad, self.t_wgrad, stream)
        # weight-gradient split sums and LayerNorm / ReZero / residual-coefficient column sums: one
        # launch (no head partials here: the State_Transfer head reduces in mep_rf_head)
        reduce_mapped(self.d_wgrad, self.d_colsum, None, None, _norm_args(self), self.redmap, stream)

    norm_fold = None   # (optimizer workspace, step, hyper) pointers: the clip's norm pass folded into the reduction

    def reduce_grid(self):
        """blocks of the backward's mep_reduce_grads launch (the optimizer's folded norm partials)"""
        return reduce_blocks(self.d_wgrad, self.d_colsum, None, self.redmap)


class RealformerRunner:
    """Flat parameters + shape-keyed plans of a State_Transfer model (or a Multi_class text chain)."""

    def __init__(self, model, spec, device):
        from .flat import FlatParams
        self.model, self.spec = model, spec
        self.device = torch.device(device)
        names = [n for n, _ in model.named_parameters()]
        self.flat = FlatParams(model, self.device, no_grad=spec.no_grad_params(names))
        self.plans = {}
        self._gen = 0
        self._live = None
        self.n_inputs = 6

    def plan(self, B, P):
        key = (int(B), int(P))
        p = self.plans.get(key)
        if p is None:
            p = RealformerPlan(self.spec, self.flat, key[0], key[1], self.device)
            self.plans[key] = p
        return p

    def plan_for(self, l):
        if self.spec.head:
            return self.plan(l.shape[0], l.shape[1])
        return self.plan(l.shape[0], 1)

    def stage(self, l, v, a, labels, lm, vm, am, umask):
        """realformer train batch order (others/realformer.py:306-309)"""
        plan = self.plan_for(l)
        plan.set_inputs(l, v, a, lm, vm, am, labels, umask)
        return plan

    def drop_p(self):
        return 0.0

    def run_forward(self, inputs):
        l, v, a, lm, vm, am = inputs
        plan = self.plan_for(l)
        plan.set_inputs(l, v, a, lm, vm, am)
        plan.forward(grad=False)
        self._gen += 1
        self._live = (plan, self._gen)
        self.token = self._gen
        return (plan.out if self.spec.head else plan.out_chain.view(l.shape[0], l.shape[1], -1)).clone()

    def run_backward(self, dout, token=None):
        plan, gen = self._live
        if token is not None and token != gen:
            raise RuntimeError('mep_amd: backward of an older forward -- call backward before the next '
                               'forward of the same shape')
        plan.backward(ext_dout=dout)
        g = self.flat.grad.clone()
        return [self.flat.view(g, n) if self.flat.has_grad[n] else None for n in self.flat.names]
