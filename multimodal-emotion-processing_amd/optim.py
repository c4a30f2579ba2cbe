"""Fused clip_grad_norm_ + AdamW / Adam over the model's flat parameter buffer.

One call = two kernel launches (global grad-norm partials; clip + update) regardless of the
number of parameter tensors -- the reference's ``nn.utils.clip_grad_norm_`` + ``optim.AdamW.step``
(cmu-mosei/run.py:368-369,398) or ``optim.Adam`` (others/realformer.py:342).  Subclasses
torch.optim.Optimizer so ``param_groups[..]['lr']`` and ``ReduceLROnPlateau`` work unchanged;
the learning rate and step count live in device memory so a captured hipGraph replays with
the current values.  Parameters without gradients (first-layer ``c``) are skipped exactly as
torch skips ``grad is None``.
"""
import ctypes

import torch

from . import _lib


class FusedAdamW(torch.optim.Optimizer):
    decoupled = True

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_norm=None):
        self.model = model
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(model.parameters(), defaults)
        self.max_norm = max_norm
        self._dev = None

    # the flat buffers are bound lazily to the model's runner (created on first GPU use)
    def _bind(self):
        runner = self.model.mep_runner()
        flat = runner.flat
        if self._dev is None or self._flat is not flat:
            dev = flat.device
            self._flat = flat
            self.exp_avg = torch.zeros_like(flat.buf)
            self.exp_avg_sq = torch.zeros_like(flat.buf)
            self.partial = torch.zeros(1024, dtype=torch.float32, device=dev)
            self.hyper = torch.zeros(8, dtype=torch.float32, device=dev)
            self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
            self.gnorm = torch.zeros(1, dtype=torch.float32, device=dev)
            self._host_hyper = None
            self._dev = dev
        return flat

    def _sync_hyper(self, max_norm=None, grad_scale=1.0):
        g = self.param_groups[0]
        mn = self.max_norm if max_norm is None else max_norm
        h = (float(g['lr']), float(g['betas'][0]), float(g['betas'][1]), float(g['eps']),
             float(g['weight_decay']), float('inf') if mn is None else float(mn), float(grad_scale))
        if h != self._host_hyper:
            self.hyper[:7].copy_(torch.tensor(h, dtype=torch.float32))
            self._host_hyper = h

    def fused_step(self, stream=None):
        """Clip + update from the flat gradient buffer (engine path; graph-capturable)."""
        flat = self._flat
        segs = (_lib.Seg * 1)(_lib.Seg(0, flat.n_grad))
        P = ctypes.c_void_p
        _lib.call('mep_clip_adam', P(flat.buf.data_ptr()), P(flat.grad.data_ptr()), P(self.exp_avg.data_ptr()),
                  P(self.exp_avg_sq.data_ptr()), ctypes.cast(segs, P), 1, flat.total, P(self.partial.data_ptr()),
                  P(self.gnorm.data_ptr()), P(self.hyper.data_ptr()), P(self.step_t.data_ptr()),
                  int(self.decoupled), stream=stream)

    @torch.no_grad()
    def step(self, closure=None):
        """torch.optim-style step: gathers ``p.grad`` into the flat buffer when they are separate
        tensors (autograd path), then runs the fused kernel."""
        loss = closure() if closure is not None else None
        flat = self._bind()
        self._sync_hyper()
        for n, p in flat.params.items():
            if not flat.has_grad[n]:
                continue
            gv = flat.view(flat.grad, n)
            if p.grad is None:
                gv.zero_()
            elif p.grad.data_ptr() != gv.data_ptr():
                gv.copy_(p.grad)
        self.fused_step()
        return loss

    def zero_grad(self, set_to_none=True):
        for p in self.model.parameters():
            p.grad = None


class FusedAdam(FusedAdamW):
    """Adam (L2 weight decay folded into the gradient; default 0) as used by realformer."""
    decoupled = False

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_norm=None):
        super().__init__(model, lr, betas, eps, weight_decay, max_norm)
