"""Drop-in mirror of robot_demo.py (the 4-model emotion demo), inference on libmep_hip.

Same class names, constructor / forward signatures and state_dict keys as the reference
(robot_demo.py:293-441): ``Unify_Dimension_Conv1d`` (five biased k=1 Conv1d projections: text 768,
visual 256 / 512 / 1024 -> D/3 each, audio 40), ``Position_Embedding``, the realformer-style
``Attention_Block`` and ``Multi_class(dim, l_len, v_len, a_len, n_heads, n_layers, ffn)`` whose
classifier reads the pooled encoder directly.  The demo configuration DIM 192 / N_HEADS 6 gives
a head dimension of 32 and an FFN width of 384 (robot_demo.py:38-43); those run on the hd = 32
attention forward (csrc/attn.hip, MEP_ATTN_HD32) and the 32-row realformer epilogue forward
(csrc/rf.hip, D = 192).

Scope: inference -- ``Multi_class.forward`` in eval mode (the reference
calls it under ``torch.no_grad()`` in ``f1_calculation`` / ``demo_output``, robot_demo.py:531-615),
``ensemble_predict`` (the 4-model mean) and ``demo_probabilities`` (demo_output's sigmoids).
Training a robot_demo model (its ``train`` with dropout 0.1) is not part of this path and raises.
"""
import math

import torch
import torch.nn as nn

from . import _autograd, _lib
from ._lib import AttnDesc, DescArray, GemmDesc, PoolDesc, RfEpiDesc, launch
from .trimodal import CHAINS, TIME_ORDER, cdiv, crows, rows

EPOCHS = 99
CLIP = 1.0
LR = 0.001
L_LEN = 25
V_LEN = 100
A_LEN = 100
DIM = 192
BATCH = 64
DROP = 0.1
FFN = 2
N_HEADS = 6
N_LAYERS = 2

EMOTIONS = ('happy', 'sad', 'angry', 'disgust', 'surprise', 'fear')
DEMO_THRESHOLDS = (0.1, 0.1, -0.1, 0.0, 0.1, 0.0)   # happ sadn ange disg surp fear (robot_demo.py:609)


def get_parameter_number(net):
    """robot_demo.py:287-290"""
    params = list(net.parameters())
    return {'Total': sum(p.numel() for p in params),
            'Trainable': sum(p.numel() for p in params if p.requires_grad)}


class Unify_Dimension_Conv1d(nn.Module):
    """robot_demo.py:293-311: biased k=1 Conv1d projections of the five feature streams."""

    def __init__(self, dim, l_dim=768, dim_1024=1024, dim_512=512, dim_256=256, a_dim=40):
        super().__init__()
        self.linguistic = nn.Conv1d(l_dim, dim, kernel_size=1)
        self.visual_1024 = nn.Conv1d(dim_1024, dim // 3, kernel_size=1)
        self.visual_512 = nn.Conv1d(dim_512, dim // 3, kernel_size=1)
        self.visual_256 = nn.Conv1d(dim_256, dim // 3, kernel_size=1)
        self.acoustic = nn.Conv1d(a_dim, dim, kernel_size=1)
        self.drop = nn.Dropout(DROP)


class Position_Embedding(nn.Module):
    """robot_demo.py:314-321"""

    def __init__(self, max_len, dim):
        super().__init__()
        self.position_embeddings = nn.Embedding(max_len, dim)
        self.len = max_len


class Attention_Block(nn.Module):
    """robot_demo.py:324-374 (the realformer block: w_qkv projections, residual scores, ReZero a / b,
    FFN, two post-LayerNorms)."""

    def __init__(self, dim, n_heads, ffn):
        super().__init__()
        self.w_qkv = nn.ModuleList([nn.Linear(dim, dim, bias=False) for _ in range(3)])
        self.n_heads = n_heads
        self.drop = nn.Dropout(DROP)
        self.proj = nn.Linear(dim, dim, bias=False)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)
        self.ffn = nn.Sequential(nn.Linear(dim, ffn * dim), nn.ReLU(), nn.Linear(ffn * dim, dim), nn.Dropout(DROP))
        self.a = nn.Parameter(torch.FloatTensor([0]), requires_grad=True)
        self.b = nn.Parameter(torch.FloatTensor([0]), requires_grad=True)
        self.c = nn.Parameter(torch.FloatTensor([0]), requires_grad=True)


class Multi_class(nn.Module):
    """robot_demo.py:377-441.  forward(l, v_256, v_512, v_1024, a, l_mask, v_mask, a_mask) -> [B, 7]
    logits, on a per-shape ``RobotPlan`` (inference)."""

    def __init__(self, dim, l_len, v_len, a_len, n_heads, n_layers, ffn):
        super().__init__()
        self.unify_dimension = Unify_Dimension_Conv1d(dim)
        self.linguistic_position = Position_Embedding(l_len, dim)
        self.visual_position = Position_Embedding(v_len, dim)
        self.acoustic_position = Position_Embedding(a_len, dim)
        self.n_layers = n_layers
        self.multimodal_blocks = nn.ModuleList([Attention_Block(dim, n_heads, ffn) for _ in range(9 * n_layers)])
        self.fully_connected = nn.Linear(dim * 6, dim)
        self.normalization = nn.LayerNorm(dim)
        self.drop = nn.Dropout(DROP)
        self.classifier = nn.Linear(dim * 6 * n_layers, 7)
        self._plans = {}

    def forward(self, l, v_256, v_512, v_1024, a, l_mask, v_mask, a_mask):
        _autograd.require_cuda(l, v_256, v_512, v_1024, a, l_mask, v_mask, a_mask)
        if self.training and DROP > 0.0:
            raise NotImplementedError('mep_amd robot_demo runs inference (eval mode); training the demo model '
                                      '(dropout 0.1) is outside this path (SURVEY.md 8(f) row 4)')
        lens = (self.linguistic_position.len, self.visual_position.len, self.acoustic_position.len)
        if (l.shape[1], v_256.shape[1], a.shape[1]) != lens:
            raise ValueError('robot_demo Multi_class adds position embeddings of lengths %s: inputs must have '
                             'exactly those lengths (robot_demo.py:392-394)' % (lens,))
        key = (int(l.shape[0]), l.device)
        plan = self._plans.get(key)
        if plan is None:
            plan = self._plans[key] = RobotPlan(self, l.shape[0], l.device)
        plan.set_inputs(l, v_256, v_512, v_1024, a, l_mask, v_mask, a_mask)
        plan.forward()
        return plan.logits.clone()


class RobotPlan:
    """Forward launch sequence of one robot_demo Multi_class at batch size B (buffers resident,
    descriptors built once; the parameters are read in place, so load_state_dict updates apply).

      unify     mep_gemm: five biased Conv1d projections (the three visual ones into column
                slices of the visual rows), each adding its position-embedding slice
      per layer mep_gemm Q / K / V projections of the 9 blocks, mep_attn_fwd (hd = 32 when
                D / H = 32), mep_rf_epi_fwd (proj, a-residual LN1, FFN, b-residual LN2) writing
                straight into the concatenated [B, T_l + T_a + T_v, 3 D n_layers] tensor
      head      mep_pool_fwd (mean | max over time), mep_gemm classifier."""

    def __init__(self, model, B, device):
        dev = torch.device(device)
        self.model, self.B, self.device = model, int(B), dev
        blk0 = model.multimodal_blocks[0]
        D = model.classifier.in_features // (6 * model.n_layers)
        H, nl, FD = blk0.n_heads, model.n_layers, blk0.ffn[0].out_features
        assert D % H == 0 and D // H in (16, 32), 'mep_attn: head dim 16 or 32'
        self.D, self.H, self.nl, self.FD = D, H, nl, FD
        u = model.unify_dimension
        self.T = {'l': model.linguistic_position.len, 'v': model.visual_position.len,
                  'a': model.acoustic_position.len}
        self.dims = {'l': u.linguistic.in_channels, 'v256': u.visual_256.in_channels,
                     'v512': u.visual_512.in_channels, 'v1024': u.visual_1024.in_channels,
                     'a': u.acoustic.in_channels}
        f32 = dict(dtype=torch.float32, device=dev)
        Tin = {'l': self.T['l'], 'v256': self.T['v'], 'v512': self.T['v'], 'v1024': self.T['v'], 'a': self.T['a']}
        self.x_in = {k: torch.zeros(B, Tin[k], d, **f32) for k, d in self.dims.items()}
        self.m_in = {m: torch.zeros(B, self.T[m], **f32) for m in 'lva'}
        self.ntok = {m: B * self.T[m] for m in 'lva'}
        self.U = {m: torch.zeros(self.ntok[m], D, **f32) for m in 'lva'}
        self.Ttot = sum(self.T.values())
        self.C = 3 * D * nl
        self.Xcat = torch.zeros(B, self.Ttot, self.C, **f32)
        self.pooled = torch.zeros(B, 2 * self.C, **f32)
        self.argmax = torch.zeros(B, self.C, dtype=torch.int32, device=dev)
        self.logits = torch.zeros(B, model.classifier.out_features, **f32)
        self.toff, t = {}, 0
        for m in TIME_ORDER:
            self.toff[m] = t
            t += self.T[m]
        self.blocks = []
        for j, (qm, km) in enumerate(CHAINS):
            for i in range(nl):
                Tq, Tk = self.T[qm], self.T[km]
                nq, nk = B * Tq, B * Tk
                b = dict(idx=len(self.blocks), j=j, i=i, qm=qm, km=km, Tq=Tq, Tk=Tk, nq=nq, nk=nk, mod=model.multimodal_blocks[nl * j + i],
                         col=((j % 3) * nl + i) * D)
                for name in ('QP', 'X', 'XP', 'Hh', 'F'):
                    b[name] = torch.zeros(nq, D, **f32)
                b['K'], b['V'] = torch.zeros(nk, D, **f32), torch.zeros(nk, D, **f32)
                b['F1'] = torch.zeros(nq, FD, **f32)
                b['estat'] = torch.zeros(nq, 4, **f32)
                b['astat'] = torch.zeros(3 * B * H * Tq, **f32)   # (max, 1/sum) per row, then the residual rows' S_prev means
                if i < nl - 1:
                    b['S'] = torch.zeros(B, H, Tq, Tk, **f32)
                self.blocks.append(b)
        self._build()

    def _out_rows(self, b):
        return rows(self.Xcat, b['Tq'], self.Ttot * self.C, self.C, self.toff[b['qm']] * self.C + b['col'])

    def _q_rows(self, b):
        if b['i'] == 0:
            return crows(self.U[b['qm']], b['Tq'], self.D)
        return self._out_rows(self.blocks[b['idx'] - 1])

    def _build(self):
        m, D, B, dev = self.model, self.D, self.B, self.device
        u = m.unify_dimension
        p = lambda t: t.data_ptr()  # noqa: E731
        g0 = dict(accumulate=0, relu=0, alpha=1.0, w_nt=1)
        ud = []
        for key, conv, pos, mod, col in (('l', u.linguistic, m.linguistic_position, 'l', 0),
                                         ('v256', u.visual_256, m.visual_position, 'v', 0),
                                         ('v512', u.visual_512, m.visual_position, 'v', D // 3),
                                         ('v1024', u.visual_1024, m.visual_position, 'v', 2 * (D // 3)),
                                         ('a', u.acoustic, m.acoustic_position, 'a', 0)):
            T, d, N = self.T[mod], self.dims[key], conv.out_channels
            # torch.cat((v_256, v_512, v_1024), 2) (robot_demo.py:310): column slices of the visual rows
            ud.append(GemmDesc(x=crows(self.x_in[key], T, d), y=rows(self.U[mod], T, T * D, D, col),
                               w=p(conv.weight), bias=p(conv.bias), table=p(pos.position_embeddings.weight) + 4 * col,
                               ntok=self.ntok[mod], N=N, K=d, ldw=d, ldt=D, **g0))
        self.d_unify = DescArray(GemmDesc, ud, dev)
        self.t_unify = max(cdiv(n, 64) for n in self.ntok.values())
        nb = dict(bias=0, table=0, N=D, K=D, ldw=D, **g0)
        self.d_proj, self.d_attn, self.d_epi, self.t_proj, self.t_attn, self.f_attn, self.t_epi = [], [], [], [], [], [], []
        hd32 = _lib.ATTN_HD32 if D // self.H == 32 else 0
        for i in range(self.nl):
            layer = [b for b in self.blocks if b['i'] == i]
            pd, ad, ed = [], [], []
            for b in layer:
                w = b['mod'].w_qkv
                pd.append(GemmDesc(x=self._q_rows(b), y=crows(b['QP'], b['Tq'], D), w=p(w[0].weight), ntok=b['nq'], **nb))
                kv = crows(self.U[b['km']], b['Tk'], D)
                pd.append(GemmDesc(x=kv, y=crows(b['K'], b['Tk'], D), w=p(w[1].weight), ntok=b['nk'], **nb))
                pd.append(GemmDesc(x=kv, y=crows(b['V'], b['Tk'], D), w=p(w[2].weight), ntok=b['nk'], **nb))
                prev = self.blocks[b['idx'] - 1] if i > 0 else None
                ad.append(AttnDesc(q=crows(b['QP'], b['Tq'], D), k=crows(b['K'], b['Tk'], D),
                                   v=crows(b['V'], b['Tk'], D), x=crows(b['X'], b['Tq'], D),
                                   mask=p(self.m_in[b['km']]), mask_sB=b['Tk'],
                                   s_prev=p(prev['S']) if prev is not None else 0, c=p(b['mod'].c),
                                   s_out=p(b['S']) if 'S' in b else 0, stats=p(b['astat']),
                                   B=B, H=self.H, Tq=b['Tq'], Tk=b['Tk']))
                mod = b['mod']
                ed.append(RfEpiDesc(q=self._q_rows(b), x=crows(b['X'], b['Tq'], D), xp=crows(b['XP'], b['Tq'], D),
                                    h=crows(b['Hh'], b['Tq'], D), f1=crows(b['F1'], b['Tq'], self.FD),
                                    f=crows(b['F'], b['Tq'], D), out=self._out_rows(b), wp=p(mod.proj.weight),
                                    w1=p(mod.ffn[0].weight), b1=p(mod.ffn[0].bias), w2=p(mod.ffn[2].weight),
                                    b2=p(mod.ffn[2].bias), ln1_w=p(mod.norm1.weight), ln1_b=p(mod.norm1.bias),
                                    ln2_w=p(mod.norm2.weight), ln2_b=p(mod.norm2.bias), a=p(mod.a), b=p(mod.b),
                                    stats=p(b['estat']), ntok=b['nq'], D=D, FD=self.FD))
            self.d_proj.append(DescArray(GemmDesc, pd, dev))
            self.t_proj.append(max(cdiv(max(b['nq'], b['nk']), 64) for b in layer))
            self.d_attn.append(DescArray(AttnDesc, ad, dev))
            geo = _lib.attn_geometry(ad)
            self.t_attn.append(geo[0])
            self.f_attn.append(geo[2] | hd32)
            self.d_epi.append(DescArray(RfEpiDesc, ed, dev))
            self.t_epi.append(max(cdiv(b['nq'], _lib.rf_epi_rows(D)) for b in layer))
        self.d_pool = DescArray(PoolDesc, [PoolDesc(x=p(self.Xcat), dx=0, pooled=p(self.pooled), dpooled=0,
                                                    argmax=p(self.argmax), B=B, T=self.Ttot, C=self.C)], dev)
        self.t_pool = B * cdiv(self.C, 32)
        F = 2 * self.C
        cls = m.classifier
        self.d_cls = DescArray(GemmDesc, [GemmDesc(x=crows(self.pooled, 1, F), y=crows(self.logits, 1, cls.out_features),
                                                   w=p(cls.weight), bias=p(cls.bias), table=0, ntok=B,
                                                   N=cls.out_features, K=F, ldw=F, **g0)], dev)

    def set_inputs(self, l, v256, v512, v1024, a, lm, vm, am):
        with torch.no_grad():
            for k, x in (('l', l), ('v256', v256), ('v512', v512), ('v1024', v1024), ('a', a)):
                self.x_in[k].copy_(x)
            for k, x in (('l', lm), ('v', vm), ('a', am)):
                self.m_in[k].copy_(x)

    def forward(self, stream=None):
        launch('mep_gemm', self.d_unify, self.t_unify, stream)
        for i in range(self.nl):
            # the Q input of layer i > 0 is layer i-1's output: projections run per layer
            launch('mep_gemm', self.d_proj[i], self.t_proj[i], stream)
            launch('mep_attn_fwd', self.d_attn[i], self.t_attn[i], stream, threads=self.f_attn[i])
            launch('mep_rf_epi_fwd', self.d_epi[i], self.t_epi[i], stream, extra=(self.D, self.FD))
        launch('mep_pool_fwd', self.d_pool, self.t_pool, stream)
        launch('mep_gemm', self.d_cls, cdiv(self.B, 64), stream)


def multi_circle_loss(y_pred, y_true):
    """robot_demo.py:444-453 (per-row loss) on libmep_hip."""
    _autograd.require_cuda(y_pred, y_true)
    return _autograd.CircleLossFunction.apply(y_pred, y_true)


def ensemble_predict(models, *inputs):
    """The 4-model ensemble of f1_calculation / demo_output: (pred_1 + ... + pred_n) / n
    (robot_demo.py:546-550, 611-615), every model in eval mode under no_grad."""
    preds = []
    with torch.no_grad():
        for mdl in models:
            mdl.eval()
            preds.append(mdl(*inputs))
    total = preds[0]
    for p in preds[1:]:
        total = total + p
    return total / len(preds)


def sigmoids(x, t):
    """robot_demo.py:594-595"""
    return 1 / (1 + math.exp(-x + t))


def demo_probabilities(pred_row, thresholds=DEMO_THRESHOLDS):
    """demo_output's printed values (robot_demo.py:616-622) before rounding: {emotion: sigmoid}."""
    row = [float(v) for v in pred_row[:6]]
    return {e: sigmoids(row[c], thresholds[c]) for c, e in enumerate(EMOTIONS)}
