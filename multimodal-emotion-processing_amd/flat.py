"""Flat parameter / gradient buffers.

Every parameter of a model is re-homed into ONE contiguous fp32 device buffer (``p.data`` becomes
a view), so the kernels address parameters by offset, the data-parallel all-reduce moves one
buffer, and clip + AdamW run as a single fused pass.  Parameters that receive gradients come
first; those that never do (the residual coefficient ``c`` of the first layer of every chain,
whose ``scores`` input is None -- cmu-mosei/run.py:243-246) are placed last so the optimizer
skips them exactly as torch skips ``grad is None`` parameters.  Names, shapes and the
state_dict order are unchanged, so reference ``.pt`` checkpoints load as before.
"""
import torch

ALIGN = 4  # floats: keep every parameter 16-byte aligned for vector loads


class FlatParams:
    def __init__(self, module, device, no_grad=(), first=None):
        """first: predicate on parameter names placed at the front of the buffer (a gradient
        bucket whose all-reduce can start before the rest of the backward; ``split`` = its end)"""
        self.device = torch.device(device)
        named = list(module.named_parameters())
        self.names = [n for n, _ in named]
        self.params = dict(named)
        no_grad = set(no_grad)
        grad = [n for n in self.names if n not in no_grad]
        if first is not None:
            grad = [n for n in grad if first(n)] + [n for n in grad if not first(n)]
        order = grad + [n for n in self.names if n in no_grad]
        self.offsets, off = {}, 0
        self.n_grad = None
        self.split = None
        for n in order:
            if first is not None and self.split is None and (n in no_grad or not first(n)):
                self.split = off
            if n in no_grad and self.n_grad is None:
                self.n_grad = off
            self.offsets[n] = off
            off += (self.params[n].numel() + ALIGN - 1) // ALIGN * ALIGN
        if self.n_grad is None:
            self.n_grad = off
        if self.split is None:
            self.split = self.n_grad
        self.total = off
        self.has_grad = {n: n not in no_grad for n in self.names}
        self.buf = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for n in order:
                p = self.params[n]
                view = self.view(self.buf, n)
                view.copy_(p.data.to(self.device, torch.float32))
                p.data = view
        self.grad = torch.zeros_like(self.buf)
        # (owner's _parameters dict, local name, parameter, its address): is_current re-checks these
        # per step instead of walking the module tree (named_parameters: ~0.4 ms of host time per
        # training step at cfg3, more than the whole step on the GPU)
        self._slots = [(m._parameters, k, p, p.data_ptr()) for _, m in module.named_modules()
                       for k, p in m._parameters.items() if p is not None]

    def view(self, buf, name):
        p = self.params[name]
        o = self.offsets[name]
        return buf[o:o + p.numel()].view(p.shape)

    def ptr(self, name):
        return self.buf.data_ptr() + 4 * self.offsets[name]

    def gptr(self, name, grad=None):
        g = self.grad if grad is None else grad
        return g.data_ptr() + 4 * self.offsets[name]

    def is_current(self, module):
        """True while every parameter still lives in this buffer: the same Parameter objects are
        registered where they were, each still a view at its offset (a ``.to()``, a
        ``load_state_dict(assign=True)`` or a re-assigned ``p.data`` / module attribute moves one)."""
        for d, k, p, ptr in self._slots:
            if d.get(k) is not p or p.data_ptr() != ptr:
                return False
        return True

    def attach_grads(self, grad=None):
        """Point every ``p.grad`` that has a gradient at its slice of the flat grad buffer."""
        g = self.grad if grad is None else grad
        for n, p in self.params.items():
            p.grad = self.view(g, n) if self.has_grad[n] else None
