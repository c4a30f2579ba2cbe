"""Drop-in mirror of the Ren-MME/run.py model + train/eval surface, running on libmep_hip.

Same class names, constructor/forward signatures and state_dict keys as the reference
(Ren-MME/run.py:151-400): ``Base_model(dim=DIM, ...)`` with its 12-argument forward
(pre_/pro_ features and masks per modality), ``multi_loss``, ``train`` (circle loss + R-Drop KL),
``valid`` and ``run``.  Differences from cmu-mosei that the shared tri-modal plan handles with
``variant='ren'``: the three unify projections share one LayerNorm ``norm1``
(run.py:164-168), the block LayerNorm is ``norm2`` with dropout(DROP) on the proj output and
after the LayerNorm (run.py:209,213), 9 classes, head LayerNorm ``norm3`` (run.py:279-292), and
float labels.  Dropout masks come from a device-side counter hash (graph-replay safe); they are
not torch's RNG stream, so runs with DROP > 0 match the reference in distribution only.
"""
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _autograd
from .runner import ModelRunner
from .trimodal import TriModalSpec

EPOCHS = 999
CLIP = 1.0
LR = 1e-3
L_LEN = 40
V_LEN = 76
A_LEN = 275
L_DIM = 768
V_DIM = 640
A_DIM = 205
DIM = 128
BATCH = 16
DROP = 0.1
FFN = 1
N_HEADS = 8
N_LAYERS = 1
N_CLASSES = 9


def get_parameter_number(net):
    """Ren-MME/run.py:153-156"""
    params = list(net.parameters())
    return {'Total': sum(p.numel() for p in params),
            'Trainable': sum(p.numel() for p in params if p.requires_grad)}


class Unify_Dimension(nn.Module):
    """Bias-free projections + ONE shared LayerNorm (Ren-MME/run.py:159-168)."""

    def __init__(self, dim):
        super().__init__()
        self.linguistic = nn.Linear(L_DIM, dim, bias=False)
        self.visual = nn.Linear(V_DIM, dim, bias=False)
        self.acoustic = nn.Linear(A_DIM, dim, bias=False)
        self.norm1 = nn.LayerNorm(dim)

    def forward(self, l, v, a):
        from .standalone import unify_norm_forward
        return unify_norm_forward(self, l, v, a)


class Attention_Block(nn.Module):
    """Residual attention block with dropout and ``norm2`` (Ren-MME/run.py:171-214)."""

    def __init__(self, dim, n_heads, ffn):
        super().__init__()
        self.n_heads = n_heads
        self.drop = nn.Dropout(DROP)
        self.proj = nn.Linear(dim, dim, bias=False)
        self.minus = nn.Linear(dim * 2, dim, bias=False)
        self.norm2 = nn.LayerNorm(dim)
        self.c = nn.Parameter(torch.FloatTensor([0]), requires_grad=True)

    def forward(self, q, k, v, mask, scores=None):
        from .standalone import block_forward
        return block_forward(self, q, k, v, mask, scores, norm=self.norm2, drop_p=self.drop.p)


class Multi_ATTN(nn.Module):
    """Nine cross-modal chains + mean/max pool + 9-way classifier (Ren-MME/run.py:217-277)."""

    def __init__(self, dim, l_len, v_len, a_len, n_heads, n_layers, ffn):
        super().__init__()
        self.unify_dimension = Unify_Dimension(dim)
        self.n_layers = n_layers
        self.multimodal_blocks = nn.ModuleList([Attention_Block(dim, n_heads, ffn) for _ in range(9 * n_layers)])
        self.classifier = nn.Linear(dim * 6 * n_layers, N_CLASSES, bias=False)

    def forward(self, l, v, a, l_mask, v_mask, a_mask):
        """Standalone entry (the training path runs this encoder inside its model's fused plan):
        HIP unify + blocks, PyTorch-ROCm concatenation / pooling / classifier."""
        from .standalone import multi_attn_forward
        return multi_attn_forward(self, l, v, a, l_mask, v_mask, a_mask)


def _pack(args):
    """Base_model's 12 forward arguments -> the plan's (prev, cur) pairs per modality."""
    (ptf, ptm, qtf, qtm, pvf, pvm, qvf, qvm, paf, pam, qaf, qam) = args
    return (ptf, qtf), (pvf, qvf), (paf, qaf), (ptm, qtm), (pvm, qvm), (pam, qam)


class Base_model(nn.Module):
    """intensity (previous utterance) + stimulation (current) encoders and the bilinear transfer
    head with norm3 (Ren-MME/run.py:279-292)."""

    def __init__(self, dim=DIM, l_len=L_LEN, v_len=V_LEN, a_len=A_LEN, n_heads=N_HEADS, n_layers=N_LAYERS,
                 ffn=FFN):
        super().__init__()
        self.intensity = Multi_ATTN(dim, l_len, v_len, a_len, n_heads, n_layers, ffn)
        self.stimulation = Multi_ATTN(dim, l_len, v_len, a_len, n_heads, n_layers, ffn)
        self.trans = nn.Parameter(torch.rand(N_CLASSES, N_CLASSES, N_CLASSES), requires_grad=True)
        self.norm3 = nn.LayerNorm(N_CLASSES)
        self.out = nn.Linear(2 * N_CLASSES, N_CLASSES)
        u = self.intensity.unify_dimension
        self._mep = dict(dim=dim, n_heads=n_heads, n_layers=n_layers,
                         dims=(u.linguistic.in_features, u.visual.in_features, u.acoustic.in_features))
        self._runner = None

    def mep_spec(self):
        c = self._mep
        return TriModalSpec(c['dim'], c['n_heads'], c['n_layers'], c['dims'], N_CLASSES, variant='ren',
                            drop_p=self.mep_drop_p())

    def mep_drop_p(self):
        """Every block's nn.Dropout shares the module-level DROP; the live value of block 0 rules."""
        return self.intensity.multimodal_blocks[0].drop.p

    def mep_runner(self, device=None):
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        r = self._runner
        if r is None or r.device != dev or not r.flat.is_current(self):
            r = ModelRunner(self, self.mep_spec(), dev, labels_float=True, n_inputs=12, pack=_pack)
            self._runner = r
        return r

    def forward(self, pre_text_feat, pre_text_mask, pro_text_feat, pro_text_mask, pre_video_feat, pre_video_mask,
                pro_video_feat, pro_video_mask, pre_audio_feat, pre_audio_mask, pro_audio_feat, pro_audio_mask):
        args = (pre_text_feat, pre_text_mask, pro_text_feat, pro_text_mask, pre_video_feat, pre_video_mask,
                pro_video_feat, pro_video_mask, pre_audio_feat, pre_audio_mask, pro_audio_feat, pro_audio_mask)
        _autograd.require_cuda(*args)
        runner = self.mep_runner(pre_text_feat.device)
        params = [runner.flat.params[n] for n in runner.flat.names]
        return _autograd.PlanFunction.apply(runner, *[t.contiguous().float() for t in args], *params)


def multi_loss(y_pred, y_true):
    """Circle loss averaged over the batch (Ren-MME/run.py:295-304), HIP kernel on CUDA tensors."""
    _autograd.require_cuda(y_pred, y_true)
    return _autograd.CircleLossFunction.apply(y_pred, y_true).mean()


def rdrop_kl(logits):
    """R-Drop term of Ren-MME/run.py:332-334 (rows 2i and 2i+1 are the same sample)."""
    kl_0 = F.kl_div(F.logsigmoid(logits[::2]), torch.sigmoid(logits[1::2]), reduction='batchmean')
    kl_1 = F.kl_div(F.logsigmoid(logits[1::2]), torch.sigmoid(logits[::2]), reduction='batchmean')
    return (kl_0 + kl_1) / 2


# ---------------------------------------------------------------------------- train / eval
def _to_device(batch, device):
    """zip(*batch) + FloatTensor(...).to(device) of run.py:316-330, via pinned host buffers."""
    out = []
    for col in zip(*batch):
        arr = np.stack([np.asarray(x, dtype=np.float32) for x in col])
        out.append(torch.from_numpy(arr).pin_memory().to(device, non_blocking=True))
    return out


def train(model, iterator, optimizer, device='cuda'):
    """One epoch (Ren-MME/run.py:307-340).  With ``mep_amd.optim.FusedAdamW`` the step (forward,
    circle loss + R-Drop KL, backward, clip, AdamW) is the fused graph-captured engine; with any
    other optimizer it follows the reference statement by statement through autograd.  Under data
    parallelism the batches are pair-preserving shares (``dp.shard_batches(loader, unit=2)``)."""
    from . import dp
    from .engine import LossSum, engine_for
    from .optim import FusedAdamW
    model.train()
    acc, count, sharded = LossSum(), 0, False
    engine = engine_for(model, optimizer, clip=CLIP, rdrop=True) if isinstance(optimizer, FusedAdamW) else None
    if engine is None and dp.world() > 1:
        raise ValueError('data-parallel training runs on the fused engine (FusedAdamW)')
    for batch in iterator:
        count += 1
        gr = dp.global_rows_of(batch)
        sharded = sharded or gr is not None
        if engine is not None and len(batch) == 0:
            acc.add(engine.step_empty(device))
            continue
        cols = _to_device(batch, device)
        args, label = cols[:12], cols[12]
        if engine is not None:
            l, v, a, lm, vm, am = _pack(args)
            loss = engine.step(l, v, a, lm, vm, am, label, global_rows=gr, row0=dp.row0_of(batch))
        else:
            optimizer.zero_grad()
            logits = model(*args)
            loss = multi_loss(logits, label) + rdrop_kl(logits)
            loss.backward()
            nn.utils.clip_grad_norm_(model.parameters(), CLIP)
            optimizer.step()
        acc.add(loss)
    return dp.epoch_mean(acc.value(), count, sharded, device)


def valid(model, iterator, device='cuda'):
    """Ren-MME/run.py:342-368: mean over batches of multi_loss (no R-Drop term); global under
    data parallelism."""
    from . import dp
    model.eval()
    epoch_loss, count, sharded = 0.0, 0, False
    with torch.no_grad():
        for batch in iterator:
            count += 1
            gr = dp.global_rows_of(batch)
            sharded = sharded or gr is not None
            if len(batch) == 0:
                continue
            cols = _to_device(batch, device)
            logits = model(*cols[:12])
            if gr is not None and dp.world() > 1:
                epoch_loss += float((_autograd.CircleLossFunction.apply(logits, cols[12]).sum() / gr).item())
            else:
                epoch_loss += float(multi_loss(logits, cols[12]).item())
    return dp.epoch_mean(epoch_loss, count, sharded, device)


def run(model, train_list, valid_list, batch_size, learning_rate, epochs, name, data_loader=None,
        log_path='.', device='cuda'):
    """Epoch driver (Ren-MME/run.py:370-402): AdamW (two groups with one lr = one group),
    ReduceLROnPlateau(0.1, patience 1), early stop after 3 epochs without improvement.
    ``data_loader(name_list, batch_size)`` is the caller's generator (the reference's reads .npy
    feature files and duplicates every sample for R-Drop; out of scope here)."""
    from torch.optim.lr_scheduler import ReduceLROnPlateau
    from .optim import FusedAdamW
    if data_loader is None:
        raise ValueError('run() needs the data_loader generator of the caller')
    from . import dp
    lead = dp.rank() == 0
    log_file = os.path.join(log_path, name + '.txt')
    if lead:
        with open(log_file, 'w') as f:
            f.write('epoch, train_loss, valid_loss\n')
    optimizer = FusedAdamW(model, lr=learning_rate)
    scheduler = ReduceLROnPlateau(optimizer, factor=0.1, patience=1)
    stop, losses = 0, []
    for epoch in range(epochs):
        train_loss = train(model, data_loader(train_list, batch_size), optimizer, device)
        valid_loss = valid(model, data_loader(valid_list, batch_size), device)
        scheduler.step(valid_loss)
        losses.append(valid_loss)
        if lead:
            with open(log_file, 'a') as f:
                f.write('\n{epoch}, {train_loss: 3.3f}, {valid_loss: 3.3f}\n'.format(
                    epoch=epoch + 1, train_loss=train_loss, valid_loss=valid_loss))
        if valid_loss == min(losses) and valid_loss > 0.009:
            stop = 0
            if lead:
                torch.save(model.state_dict(), os.path.join(log_path, name + '_' + str(valid_loss)[:4] + '.pt'))
        else:
            stop += 1
            if stop >= 3:
                break
