"""Drop-in mirror of the cmu-mosei/run.py model + train/eval surface, running on libmep_hip.

Same class names, constructor signatures, forward signatures and state_dict keys as the
reference (cmu-mosei/run.py:201-420), so ``Concat_Trans(dim=DIM, l_len=L_LEN, ...)``, reference
``.pt`` checkpoints, ``optim.AdamW(model.parameters())``, ``multi_circle_loss``, ``train``,
``valid`` and ``run`` are used exactly as in the reference script.  On CUDA tensors the whole
``Concat_Trans`` forward/backward executes as the fused HIP plan (trimodal.py); there is no CPU
execution path (use the oracle for CPU).

Module constants mirror run.py:28-42 and are read at construction time, as the reference's
module globals are.
"""
import os

import numpy as np
import torch
import torch.nn as nn

from . import _autograd
from .runner import ModelRunner
from .trimodal import TriModalSpec

EPOCHS = 999
CLIP = 1.0
LR = 0.001
L_LEN = 20
V_LEN = 100
A_LEN = 200
L_DIM = 300
V_DIM = 35
A_DIM = 74
DIM = 96
BATCH = 64
DROP = 0.0
FFN = 1
N_HEADS = 6
N_LAYERS = 1
N_CLASSES = 7


def get_parameter_number(net):
    """cmu-mosei/run.py:201-204"""
    params = list(net.parameters())
    return {'Total': sum(p.numel() for p in params),
            'Trainable': sum(p.numel() for p in params if p.requires_grad)}


class Unify_Dimension(nn.Module):
    """Three bias-free projections to the shared width (cmu-mosei/run.py:207-214).  Executed
    inside the owning model's plan (one grouped MFMA GEMM launch)."""

    def __init__(self, dim):
        super().__init__()
        self.linguistic = nn.Linear(L_DIM, dim, bias=False)
        self.visual = nn.Linear(V_DIM, dim, bias=False)
        self.acoustic = nn.Linear(A_DIM, dim, bias=False)

    def forward(self, l, v, a):
        from .standalone import unify_forward
        return unify_forward(self, l, v, a)


class Attention_Block(nn.Module):
    """Residual attention block without Q/K/V projection (cmu-mosei/run.py:217-262)."""

    def __init__(self, dim, n_heads, ffn):
        super().__init__()
        self.n_heads = n_heads
        self.drop = nn.Dropout(DROP)
        self.proj = nn.Linear(dim, dim, bias=False)
        self.minus = nn.Linear(dim * 2, dim, bias=False)
        self.norm1 = nn.LayerNorm(dim)
        self.c = nn.Parameter(torch.FloatTensor([0]), requires_grad=True)

    def forward(self, q, k, v, mask, scores=None):
        from .standalone import block_forward
        return block_forward(self, q, k, v, mask, scores, norm=self.norm1, drop_p=self.drop.p)


class Multi_ATTN(nn.Module):
    """Nine cross-modal chains + mean/max pool + classifier (cmu-mosei/run.py:265-319)."""

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


class Concat_Trans(nn.Module):
    """Previous/current utterance encoders + bilinear transfer head (cmu-mosei/run.py:321-339)."""

    def __init__(self, dim, l_len, v_len, a_len, n_heads, n_layers, ffn):
        super().__init__()
        self.intensity = Multi_ATTN(dim, l_len, v_len, a_len, n_heads, n_layers, ffn)
        self.stimulation = Multi_ATTN(dim, l_len, v_len, a_len, n_heads, n_layers, ffn)
        self.trans = nn.Parameter(torch.rand(N_CLASSES, N_CLASSES, N_CLASSES), requires_grad=True)
        self.norm1 = nn.LayerNorm(N_CLASSES)
        self.out = nn.Linear(2 * N_CLASSES, N_CLASSES)
        self._mep = dict(dim=dim, n_heads=n_heads, n_layers=n_layers,
                         dims=(self.intensity.unify_dimension.linguistic.in_features,
                               self.intensity.unify_dimension.visual.in_features,
                               self.intensity.unify_dimension.acoustic.in_features))
        self._runner = None

    def mep_spec(self):
        c = self._mep
        return TriModalSpec(c['dim'], c['n_heads'], c['n_layers'], c['dims'], N_CLASSES, variant='cmu')

    def mep_runner(self, device=None):
        """The model's HIP runtime (flat parameters + plans); created on first GPU use."""
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        r = self._runner
        if r is None or r.device != dev or not r.flat.is_current(self):
            r = ModelRunner(self, self.mep_spec(), dev)
            self._runner = r
        return r

    def forward(self, l, v, a, l_mask, v_mask, a_mask):
        _autograd.require_cuda(l, v, a, l_mask, v_mask, a_mask)
        runner = self.mep_runner(l.device)
        params = [runner.flat.params[n] for n in runner.flat.names]
        args = [t.contiguous().float() for t in (l, v, a, l_mask, v_mask, a_mask)]
        return _autograd.PlanFunction.apply(runner, *args, *params)


def multi_circle_loss(y_pred, y_true):
    """Per-row multi-label circle loss (cmu-mosei/run.py:342-351), HIP kernel on CUDA tensors."""
    _autograd.require_cuda(y_pred, y_true)
    return _autograd.CircleLossFunction.apply(y_pred, y_true)


# ---------------------------------------------------------------------------- train / eval
def _to_device(batch, device):
    """zip(*batch) + tensor construction of run.py:361-363, via pinned host buffers (batches from
    ``batching.cmu_data_loader`` are already on the device and pass through)."""
    from .batching import DeviceBatch
    if isinstance(batch, DeviceBatch):
        return list(batch)
    cols = list(zip(*batch))
    out = []
    for i, col in enumerate(cols):
        arr = np.stack([np.asarray(x) for x in col])
        dt = torch.int64 if i == 6 else torch.float32
        out.append(torch.from_numpy(arr).to(dt).pin_memory().to(device, non_blocking=True))
    return out


def train(model, iterator, optimizer, device='cuda'):
    """One epoch (cmu-mosei/run.py:354-372).  With an ``mep_amd.optim.FusedAdamW`` optimizer the
    whole step (forward, loss, backward, clip, AdamW) runs as the fused engine; with any other
    optimizer it follows the reference statement by statement through autograd.  Under data
    parallelism (mep_amd.dp) the batches are this rank's shares of the global batches and the
    returned epoch loss is the global one, identical on every rank."""
    from . import dp
    from .engine import LossSum, engine_for
    from .optim import FusedAdamW
    model.train()
    acc, count, sharded = LossSum(), 0, False
    engine = engine_for(model, optimizer, clip=CLIP) if isinstance(optimizer, FusedAdamW) else None
    if engine is None and dp.world() > 1:
        raise ValueError('data-parallel training runs on the fused engine (FusedAdamW)')
    for batch in iterator:
        count += 1
        gr = dp.global_rows_of(batch)
        sharded = sharded or gr is not None
        if engine is not None and len(batch) == 0:      # empty share of a ragged global batch
            acc.add(engine.step_empty(device))
            continue
        l, v, a, lm, vm, am, label = _to_device(batch, device)
        if engine is not None:
            loss = engine.step(l, v, a, lm, vm, am, label, global_rows=gr, row0=dp.row0_of(batch))
        else:
            optimizer.zero_grad()
            logits = model(l, v, a, lm, vm, am)
            loss = multi_circle_loss(logits, label).mean()
            loss.backward()
            nn.utils.clip_grad_norm_(model.parameters(), CLIP)
            optimizer.step()
        acc.add(loss)
    return dp.epoch_mean(acc.value(), count, sharded, device)


def valid(model, iterator, device='cuda'):
    """cmu-mosei/run.py:375-390 -> (sum of batch losses, batches, mean); global under data
    parallelism (each rank adds its share of every global batch's mean)."""
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
            l, v, a, lm, vm, am, label = _to_device(batch, device)
            logits = model(l, v, a, lm, vm, am)
            rl = multi_circle_loss(logits, label)
            epoch_loss += float((rl.sum() / gr if gr is not None and dp.world() > 1 else rl.mean()).item())
    mean = dp.epoch_mean(epoch_loss, count, sharded, device)
    return mean * count, count, mean


def run(model, train_list, valid_list, label_dict, batch_size, learning_rate, epochs, log_name,
        data_loader=None, log_dir='.', device='cuda'):
    """Epoch driver (cmu-mosei/run.py:393-420): AdamW, ReduceLROnPlateau(0.1, 4), early stop
    after 9 epochs without improvement, best checkpoint saved under the reference's file name.
    ``data_loader(name_list, label_dict, batch_size)`` is the caller's batch generator (the
    reference's reads CMU-MOSEI .csd files, which are outside this framework's scope)."""
    from torch.optim.lr_scheduler import ReduceLROnPlateau
    from .optim import FusedAdamW
    if data_loader is None:
        raise ValueError('run() needs the data_loader generator of the caller')
    from . import dp
    lead = dp.rank() == 0                   # data parallelism: one log / checkpoint writer
    log_file = os.path.join(log_dir, log_name + '.txt')
    if lead:
        with open(log_file, 'w') as f:
            f.write('epoch, train_loss, valid_loss\n')
    optimizer = FusedAdamW(model, lr=learning_rate)
    scheduler = ReduceLROnPlateau(optimizer, factor=0.1, patience=4)
    stop, losses = 0, []
    for epoch in range(epochs):
        train_loss = train(model, data_loader(train_list, label_dict, batch_size), optimizer, device)
        _, _, valid_loss = valid(model, data_loader(valid_list, label_dict, batch_size), device)
        scheduler.step(valid_loss)           # the same global valid loss on every rank
        losses.append(valid_loss)
        if lead:
            with open(log_file, 'a') as f:
                f.write('\n{epoch},{train_loss: 2.2f},{valid_loss: 2.2f}\n'.format(
                    epoch=epoch + 1, train_loss=train_loss, valid_loss=valid_loss))
        if valid_loss == min(losses) and valid_loss > 0.009:
            stop = 0
            if lead:
                torch.save(model.state_dict(), os.path.join(log_dir, log_name + '_' + str(valid_loss)[:4] + '.pt'))
        else:
            stop += 1
            if stop >= 9:
                break
