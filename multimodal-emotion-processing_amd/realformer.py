"""Drop-in mirror of others/realformer.py (State_Transfer family), running on libmep_hip.

Same class names, constructor/forward signatures and state_dict keys as the reference
(others/realformer.py:128-360): ``State_Transfer(l_dim, v_dim, a_dim, dim, l_len, v_len, a_len,
n_heads, n_layers, ffn)`` over ``[B, P, T, d]`` utterance windows, ``multi_circle_loss``,
``train`` / ``valid`` / ``run`` (Adam, circle loss masked by the utterance mask).  As in the
reference, ``Attention_Block`` reads the module constant FFN for its hidden width (the ``ffn``
constructor argument is accepted and unused, realformer.py:154-168,221).

``encode_chain`` runs the BASELINE cfg2 workload ("text encoder, realformer attention only"):
Conv1d unify of the text features + position embedding + ``n_layers`` residual blocks of chain
(l, l) = ``multimodal_blocks[0 .. n_layers-1]`` (realformer.py:224-233).
"""
import os

import numpy as np
import torch
import torch.nn as nn

from . import _autograd
from .rf_plan import RealformerRunner, RealformerSpec

L_DIM = 300
V_DIM = 35
A_DIM = 74
L_LEN = 50
V_LEN = 50
A_LEN = 50
CLIP = 1.0
EPOCHS = 99
BATCH = 64
DIM = 96
N_HEADS = 6
FFN = 2
N_LAYERS = 2
LR = 0.001
DROP = 0.0
P_LEN = 6


def get_parameter_number(net):
    """others/realformer.py:128-131"""
    params = list(net.parameters())
    return {'Total': sum(p.numel() for p in params),
            'Trainable': sum(p.numel() for p in params if p.requires_grad)}


class Unify_Dimension_Conv1d(nn.Module):
    """k=1 Conv1d projections (realformer.py:133-143) == bias-free Linear on the feature axis."""

    def __init__(self, l_dim, v_dim, a_dim, dim):
        super().__init__()
        self.linguistic = nn.Conv1d(l_dim, dim, kernel_size=1, bias=False)
        self.visual = nn.Conv1d(v_dim, dim, kernel_size=1, bias=False)
        self.acoustic = nn.Conv1d(a_dim, dim, kernel_size=1, bias=False)
        self.drop = nn.Dropout(DROP)

    def forward(self, l, v, a):
        from .standalone import linear_nobias
        if self.training and self.drop.p > 0.0:
            raise NotImplementedError('realformer dropout: the reference runs DROP = 0')
        return tuple(linear_nobias(x, conv.weight[:, :, 0])
                     for x, conv in ((l, self.linguistic), (v, self.visual), (a, self.acoustic)))


class Position_Embedding(nn.Module):
    """Learned absolute positions (realformer.py:145-152): returns the table broadcast over the
    batch (a view; the fused plan adds it inside the unify GEMM)."""

    def __init__(self, max_len, dim):
        super().__init__()
        self.position_embeddings = nn.Embedding(max_len, dim)
        self.len = max_len

    def forward(self, x):
        w = self.position_embeddings.weight
        return w.unsqueeze(0).expand(x.size()[0], self.len, w.shape[1])


class Attention_Block(nn.Module):
    """RealFormer residual-attention block (realformer.py:154-209)."""

    def __init__(self, dim, n_heads):
        super().__init__()
        self.w_qkv = nn.ModuleList([nn.Linear(dim, dim, bias=False) for _ in range(3)])
        self.n_heads = n_heads
        self.drop = nn.Dropout(DROP)
        self.proj = nn.Linear(dim, dim, bias=False)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)
        self.ffn = nn.Sequential(nn.Linear(dim, FFN * dim), nn.ReLU(), nn.Linear(FFN * dim, dim), nn.Dropout(DROP))
        self.a = nn.Parameter(torch.FloatTensor([0]), requires_grad=True)
        self.b = nn.Parameter(torch.FloatTensor([0]), requires_grad=True)
        self.c = nn.Parameter(torch.FloatTensor([0]), requires_grad=True)

    def forward(self, q, k, v, mask, scores=None):
        from .standalone import rf_block_forward
        return rf_block_forward(self, q, k, v, mask, scores)


class Multi_class(nn.Module):
    """Conv1d unify + positions + 9 residual chains x n_layers + pool + FC/LN/ReLU
    (realformer.py:211-264)."""

    def __init__(self, l_dim, v_dim, a_dim, dim, l_len, v_len, a_len, n_heads, n_layers, ffn):
        super().__init__()
        self.unify_dimension = Unify_Dimension_Conv1d(l_dim, v_dim, a_dim, dim)
        self.linguistic_position = Position_Embedding(l_len, dim)
        self.visual_position = Position_Embedding(v_len, dim)
        self.acoustic_position = Position_Embedding(a_len, dim)
        self.n_layers = n_layers
        self.multimodal_blocks = nn.ModuleList([Attention_Block(dim, n_heads) for _ in range(9 * n_layers)])
        self.fully_connected = nn.Linear(dim * 6, dim)
        self.normalization = nn.LayerNorm(dim)
        self.drop = nn.Dropout(DROP)
        self._mep = dict(dim=dim, n_heads=n_heads, n_layers=n_layers, dims=(l_dim, v_dim, a_dim),
                         T=(l_len, v_len, a_len))
        self._chain_runner = None

    def forward(self, l, v, a, l_mask, v_mask, a_mask):
        """Standalone entry (the training path runs this encoder inside its model's fused plan):
        HIP unify + blocks, PyTorch-ROCm concatenation / pooling / FC + LayerNorm + ReLU."""
        from .standalone import multi_class_forward
        return multi_class_forward(self, l, v, a, l_mask, v_mask, a_mask)

    def mep_chain_runner(self, n_layers, device):
        c = self._mep
        r = self._chain_runner
        if r is None or r.device != torch.device(device) or r.spec.nl != n_layers or not r.flat.is_current(self):
            FD = self.multimodal_blocks[0].ffn[0].out_features
            spec = RealformerSpec(c['dim'], c['n_heads'], n_layers, FD, c['dims'], c['T'], prefix='',
                                  chains=(('l', 'l'),), head=False)   # multimodal_blocks[0 .. n_layers-1]
            r = RealformerRunner(self, spec, device)
            self._chain_runner = r
        return r


class State_Transfer(nn.Module):
    """Shared Multi_class encoder over P utterances + sigmoid/tanh state transfer
    (realformer.py:266-286).  Inputs [B, P, T, d] and masks [B, P, T]; returns [B, P, 6]."""

    def __init__(self, l_dim, v_dim, a_dim, dim, l_len, v_len, a_len, n_heads, n_layers, ffn):
        super().__init__()
        self.feature = Multi_class(l_dim=l_dim, v_dim=v_dim, a_dim=a_dim, dim=dim, l_len=l_len, v_len=v_len,
                                   a_len=a_len, n_heads=n_heads, n_layers=n_layers, ffn=ffn)
        self.classifier = nn.Linear(dim, 6 * 2)
        self.trans = nn.Parameter(torch.rand(6, 6), requires_grad=True)
        self._runner = None

    def mep_spec(self):
        c = self.feature._mep
        FD = self.feature.multimodal_blocks[0].ffn[0].out_features
        return RealformerSpec(c['dim'], c['n_heads'], c['n_layers'], FD, c['dims'], c['T'], prefix='feature.')

    def mep_runner(self, device=None):
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        r = self._runner
        if r is None or r.device != dev or not r.flat.is_current(self):
            r = RealformerRunner(self, self.mep_spec(), dev)
            self._runner = r
        return r

    def forward(self, l, v, a, l_mask, v_mask, a_mask):
        args = (l, v, a, l_mask, v_mask, a_mask)
        _autograd.require_cuda(*args)
        if self.training and any(m.p > 0.0 for m in self.modules() if isinstance(m, nn.Dropout)):
            raise NotImplementedError('realformer dropout: the reference runs DROP = 0 (realformer.py:37)')
        runner = self.mep_runner(l.device)
        params = [runner.flat.params[n] for n in runner.flat.names]
        return _autograd.PlanFunction.apply(runner, *[t.contiguous().float() for t in args], *params)


def encode_chain(model, l, l_mask, n_layers=N_LAYERS):
    """BASELINE cfg2 text encoder: ``model`` is a Multi_class; l [B, T, l_dim], l_mask [B, T] ->
    [B, T, dim] after Conv1d unify + position embedding + multimodal_blocks[0 .. n_layers-1]
    (realformer.py:224-233), differentiable w.r.t. every parameter it uses."""
    _autograd.require_cuda(l, l_mask)
    runner = model.mep_chain_runner(n_layers, l.device)
    params = [runner.flat.params[n] for n in runner.flat.names]
    z = torch.zeros(0, device=l.device)
    return _autograd.PlanFunction.apply(runner, l.contiguous().float(), z, z, l_mask.contiguous().float(), z, z,
                                        *params)


def multi_circle_loss(y_pred, y_true):
    """realformer.py:289-298 -> per-(row, utterance) loss [..., ]; HIP kernel on CUDA tensors."""
    _autograd.require_cuda(y_pred, y_true)
    lead = y_pred.shape[:-1]
    nc = y_pred.shape[-1]
    out = _autograd.CircleLossFunction.apply(y_pred.reshape(-1, nc), y_true.reshape(-1, nc))
    return out.reshape(lead)


# ---------------------------------------------------------------------------- train / eval
def _to_device(batch, device):
    """zip(*batch) + torch.cuda.FloatTensor / LongTensor of realformer.py:307-309 (batches from
    ``batching.rf_data_loader`` are already on the device and pass through)."""
    from .batching import DeviceBatch
    if isinstance(batch, DeviceBatch):
        return list(batch)
    out = []
    for i, col in enumerate(zip(*batch)):
        arr = np.stack([np.asarray(x) for x in col])
        dt = torch.int64 if i in (3, 7) else torch.float32
        out.append(torch.from_numpy(arr).to(dt).pin_memory().to(device, non_blocking=True))
    return out


def train(model, iterator, optimizer, device='cuda'):
    """One epoch (realformer.py:300-318).  With ``mep_amd.optim.FusedAdam`` the step (forward,
    masked circle loss, backward, clip, Adam) is the fused graph-captured engine.  Under data
    parallelism (mep_amd.dp) the batches are this rank's shares of the global batches."""
    from . import dp
    from .engine import LossSum, engine_for
    from .optim import FusedAdamW
    model.train()
    acc, count, sharded = LossSum(), 0, False
    engine = engine_for(model, optimizer, clip=CLIP) if isinstance(optimizer, FusedAdamW) else None
    if engine is None and dp.world() > 1:
        raise ValueError('data-parallel training runs on the fused engine (FusedAdam)')
    for batch in iterator:
        count += 1
        gr = dp.global_rows_of(batch)
        sharded = sharded or gr is not None
        if engine is not None and len(batch) == 0:
            acc.add(engine.step_empty(device))
            continue
        l, v, a, label, lm, vm, am, mask = _to_device(batch, device)
        if engine is not None:
            loss = engine.step(l, v, a, label, lm, vm, am, mask, global_rows=gr, row0=dp.row0_of(batch))
        else:
            optimizer.zero_grad()
            logits = model(l, v, a, lm, vm, am)
            loss = (multi_circle_loss(logits, label) * mask).mean()
            loss.backward()
            nn.utils.clip_grad_norm_(model.parameters(), CLIP)
            optimizer.step()
        acc.add(loss)
    return dp.epoch_mean(acc.value(), count, sharded, device)


def valid(model, iterator, device='cuda'):
    """realformer.py:320-334 -> (sum of batch losses, batches, mean); global under data
    parallelism."""
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
            l, v, a, label, lm, vm, am, mask = _to_device(batch, device)
            logits = model(l, v, a, lm, vm, am)
            masked = multi_circle_loss(logits, label) * mask
            if gr is not None and dp.world() > 1:
                epoch_loss += float((masked.sum() / (gr * masked.shape[1])).item())
            else:
                epoch_loss += float(masked.mean().item())
    mean = dp.epoch_mean(epoch_loss, count, sharded, device)
    return mean * count, count, mean


def run(model, data_set, train_list, valid_list, batch_size, learning_rate, epochs, name, data_loader=None,
        log_dir='.', device='cuda'):
    """Epoch driver (realformer.py:336-360): Adam, ReduceLROnPlateau(0.1, patience 2), early stop
    after 4 epochs without improvement.  ``data_loader(data_set, name_list, batch_size)`` is the
    caller's generator (the reference's reads CMU-MOSEI .csd files; out of scope here)."""
    from torch.optim.lr_scheduler import ReduceLROnPlateau
    from .optim import FusedAdam
    if data_loader is None:
        raise ValueError('run() needs the data_loader generator of the caller')
    from . import dp
    lead = dp.rank() == 0
    log_file = os.path.join(log_dir, name + '.txt')
    if lead:
        with open(log_file, 'w') as f:
            f.write('epoch, train_loss, valid_loss\n')
    optimizer = FusedAdam(model, lr=learning_rate)
    scheduler = ReduceLROnPlateau(optimizer, factor=0.1, patience=2)
    stop, losses = 0, []
    for epoch in range(epochs):
        train_loss = train(model, data_loader(data_set, train_list, batch_size), optimizer, device)
        _, _, valid_loss = valid(model, data_loader(data_set, valid_list, batch_size), device)
        scheduler.step(valid_loss)
        losses.append(valid_loss)
        if lead:
            with open(log_file, 'a') as f:
                f.write('\n{epoch},{train_loss: 2.2f},{valid_loss: 2.2f}\n'.format(
                    epoch=epoch + 1, train_loss=train_loss, valid_loss=valid_loss))
        if valid_loss == min(losses):
            stop = 0
            if lead:
                torch.save(model.state_dict(), os.path.join(log_dir, name + '_' + str(valid_loss)[:4] + '.pt'))
        else:
            stop += 1
            if stop >= 4:
                break
