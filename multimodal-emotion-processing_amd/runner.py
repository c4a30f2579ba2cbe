"""Per-model runtime state: the flat parameter buffer and the shape-keyed plan cache.

``ModelRunner`` is attached lazily to a drop-in model the first time it runs on a GPU.  It
re-homes the parameters into a ``FlatParams`` buffer, builds one ``TriModalPlan`` per input
shape (batch, T_l, T_v, T_a) and serves both the autograd path (``run_forward`` /
``run_backward``) and the fused training engine (engine.py).
"""
import torch

from .flat import FlatParams
from .trimodal import TriModalPlan


class ModelRunner:
    def __init__(self, model, spec, device, labels_float=False, n_inputs=6, pack=None):
        """``pack`` maps the model's forward arguments (``n_inputs`` tensors) to the plan's
        (l, v, a, l_mask, v_mask, a_mask); None = they already are in that order."""
        self.model = model
        self.n_inputs = n_inputs
        self.pack = pack
        self.spec = spec
        self.device = torch.device(device)
        self.labels_float = labels_float
        # gradient bucket A first (the block weights, LayerNorms and the fusion head: ready after the
        # last epilogue backward), so a data-parallel all-reduce of it overlaps the attention
        # backward and the unify weight gradients (engine.py)
        self.flat = FlatParams(model, self.device, no_grad=spec.no_grad_params(), first=spec.bucket_a)
        self.plans = {}
        # dropout state shared by every plan of this model: {seed, row0}.  One seed stream per
        # model (not per plan shape), advanced once per training step -- also by an empty
        # data-parallel share -- so every rank holds the same seed at every step
        self.seed_state = torch.zeros(2, dtype=torch.int64, device=self.device)
        self._gen = 0
        self._live = None

    def bf16(self):
        """The bf16 path (csrc MEP_PREC_BF16) runs when the model is called under
        ``torch.autocast(device_type='cuda', dtype=torch.bfloat16)`` -- the way reference-side code
        asks for bf16 -- or when ``model.mep_precision == 'bf16'``; otherwise the fp32 path."""
        if getattr(self.model, 'mep_precision', 'fp32') == 'bf16':
            return True
        return torch.is_autocast_enabled('cuda') and torch.get_autocast_dtype('cuda') == torch.bfloat16

    def plan(self, B, T, bf16=None):
        bf16 = self.bf16() if bf16 is None else bool(bf16)
        key = (int(B),) + tuple(int(t) for t in T) + (bf16,)
        p = self.plans.get(key)
        if p is None:
            p = TriModalPlan(self.spec, self.flat, key[0], key[1:4], self.device, self.labels_float, bf16=bf16,
                             seed_state=self.seed_state)
            self.plans[key] = p
        return p

    def plan_for(self, l, v, a):
        """Plan for a batch given either as [B, 2, T, d] (prev, cur) tensors (cmu-mosei) or as
        (prev, cur) pairs of [B, T, d] tensors (Ren-MME's separate pre_/pro_ arguments)."""
        def bt(x):
            x0 = x[0] if isinstance(x, (tuple, list)) else x
            return x0.shape[0], x0.shape[-2]
        B = bt(l)[0]
        return self.plan(B, (bt(l)[1], bt(v)[1], bt(a)[1]))

    def stage(self, l, v, a, lm, vm, am, labels):
        """Plan for the batch's shape with the batch copied into its resident buffers."""
        plan = self.plan_for(l, v, a)
        plan.set_inputs(l, v, a, lm, vm, am, labels)
        return plan

    def drop_p(self):
        """Dropout probability of the current mode (the model's live nn.Dropout p in train mode)."""
        if not self.model.training:
            return 0.0
        fn = getattr(self.model, 'mep_drop_p', None)
        return float(fn()) if fn is not None else self.spec.drop_p

    # ------------------------------------------------------------ autograd path
    def run_forward(self, inputs):
        l, v, a, lm, vm, am = self.pack(inputs) if self.pack is not None else inputs
        plan = self.plan_for(l, v, a)
        p = self.drop_p()
        plan.set_dropout(p)
        if p > 0.0:
            plan.set_row0(0)
            plan.advance_seed()
        plan.set_inputs(l, v, a, lm, vm, am)
        plan.forward(grad=False)
        self._gen += 1
        self._live = (plan, self._gen)
        self.token = self._gen
        return plan.logits.clone()

    def run_backward(self, dlogits, token=None):
        plan, gen = self._live
        if token is not None and token != gen:
            raise RuntimeError('mep_amd: backward of an older forward -- this plan keeps the '
                               'activations of the latest forward only; call backward before the next '
                               'forward of the same shape')
        plan.backward(ext_dlogits=dlogits)
        g = self.flat.grad.clone()
        return [self.flat.view(g, n) if self.flat.has_grad[n] else None for n in self.flat.names]
