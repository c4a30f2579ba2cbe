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
            # [0, 1016) norm partials, [1016, 1018) step scalars, [1024, ..) the partials of a
            # mep_reduce_grads launch that folded the norm pass in (TrainEngine, single process)
            self.partial = torch.zeros(1024 + self.MAX_EXT, dtype=torch.float32, device=dev)
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

    MAX_EXT = 1 << 16   # largest folded-norm launch (mep_reduce_grads blocks)

    def norm_fold_ptrs(self):
        """(workspace, step, hyper) device pointers a plan's mep_reduce_grads writes the folded
        norm partials and step scalars to"""
        return (self.partial.data_ptr(), self.step_t.data_ptr(), self.hyper.data_ptr())

    def fused_step(self, stream=None, n_ext=0):
        """Clip + update from the flat gradient buffer (engine path; graph-capturable).  n_ext > 0:
        the backward's reduction already wrote n_ext norm partials and advanced the step."""
        assert 0 <= n_ext <= self.MAX_EXT
        flat = self._flat
        segs = (_lib.Seg * 1)(_lib.Seg(0, flat.n_grad))
        P = ctypes.c_void_p
        _lib.call('mep_clip_adam_ext', P(flat.buf.data_ptr()), P(flat.grad.data_ptr()), P(self.exp_avg.data_ptr()),
                  P(self.exp_avg_sq.data_ptr()), ctypes.cast(segs, P), 1, flat.total, P(self.partial.data_ptr()),
                  P(self.gnorm.data_ptr()), P(self.hyper.data_ptr()), P(self.step_t.data_ptr()),
                  int(self.decoupled), int(n_ext), stream=stream)

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

    # ------------------------------------------------------------------ checkpoint / resume
    # SURVEY 8(f) row 3.  The reference saves only the model (cmu-mosei/run.py:415); optimizer
    # state is kept here in torch.optim.AdamW / Adam's own state_dict layout (state keyed by the
    # index in model.parameters(), 'step' / 'exp_avg' / 'exp_avg_sq' shaped like each parameter;
    # parameters that never get a gradient carry no state), so a checkpoint round-trips through
    # torch.save and loads into either optimizer.
    def _torch_cls(self):
        return torch.optim.AdamW if self.decoupled else torch.optim.Adam

    def state_dict(self):
        g = self.param_groups[0]
        ref = self._torch_cls()([torch.zeros(1)], lr=g['lr'], betas=g['betas'], eps=g['eps'],
                                weight_decay=g['weight_decay'])
        group = dict(ref.param_groups[0])
        names = [n for n, _ in self.model.named_parameters()]
        group['params'] = list(range(len(names)))
        state = {}
        if self._dev is not None:
            flat = self._flat
            steps = int(self.step_t.item())
            if steps > 0:
                for i, n in enumerate(names):
                    if flat.has_grad[n]:
                        state[i] = {'step': torch.tensor(float(steps)),
                                    'exp_avg': flat.view(self.exp_avg, n).detach().cpu().clone(),
                                    'exp_avg_sq': flat.view(self.exp_avg_sq, n).detach().cpu().clone()}
        return {'state': state, 'param_groups': [group]}

    @torch.no_grad()
    def load_state_dict(self, state_dict):
        groups = state_dict['param_groups']
        if len(groups) != 1:
            raise ValueError('FusedAdamW.load_state_dict: expected one parameter group, got %d' % len(groups))
        names = [n for n, _ in self.model.named_parameters()]
        if len(groups[0]['params']) != len(names):
            raise ValueError('FusedAdamW.load_state_dict: %d parameters in the checkpoint, %d in the model'
                             % (len(groups[0]['params']), len(names)))
        for k in ('lr', 'betas', 'eps', 'weight_decay'):
            if k in groups[0]:
                self.param_groups[0][k] = groups[0][k]
        flat = self._bind()
        state = state_dict['state']
        idx = {p: i for i, p in enumerate(groups[0]['params'])}
        steps = set()
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        for i, n in enumerate(names):
            s = state.get(groups[0]['params'][i], state.get(i)) if idx else None
            if s is None:
                continue
            if not flat.has_grad[n]:
                raise ValueError('FusedAdamW.load_state_dict: state for %s, which never gets a gradient' % n)
            flat.view(self.exp_avg, n).copy_(s['exp_avg'])
            flat.view(self.exp_avg_sq, n).copy_(s['exp_avg_sq'])
            steps.add(int(float(s['step'])))
        if len(steps) > 1:
            raise ValueError('FusedAdamW.load_state_dict: parameters at different step counts %s' % sorted(steps))
        self.step_t.fill_(steps.pop() if steps else 0)
        self._host_hyper = None


class FusedAdam(FusedAdamW):
    """Adam (L2 weight decay folded into the gradient; default 0) as used by realformer."""
    decoupled = False

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_norm=None):
        super().__init__(model, lr, betas, eps, weight_decay, max_norm)
