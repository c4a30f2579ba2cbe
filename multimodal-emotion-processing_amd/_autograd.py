"""Bridge between the drop-in nn.Modules and the HIP execution plans.

``model(...)`` on CUDA tensors runs the whole encoder pair + head forward as ONE autograd node:
forward launches the plan's kernels and returns logits; backward takes dlogits, launches the
plan's backward (which writes every parameter gradient into the flat gradient buffer) and hands
autograd a private copy of each parameter's slice, so ``loss.backward()``, gradient
accumulation, ``clip_grad_norm_`` and any torch optimizer behave exactly as with the reference.
There is no CPU path: CPU tensors raise (the CPU restatement lives in the test-only oracle).
"""
import ctypes

import torch

from . import _lib


def require_cuda(*tensors):
    for t in tensors:
        if torch.is_tensor(t) and not t.is_cuda:
            raise RuntimeError('mep_amd runs on the GPU through libmep_hip (HIP/gfx950); got a CPU tensor. '
                               'There is no CPU fallback in the product path.')


class PlanFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, runner, *args):
        # args = inputs..., then every parameter (so autograd routes their grads here)
        logits = runner.run_forward(args[:runner.n_inputs])
        ctx.runner = runner
        ctx.token = runner.token
        return logits

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dlogits):
        runner = ctx.runner
        grads = runner.run_backward(dlogits.contiguous(), ctx.token)
        return (None,) + (None,) * runner.n_inputs + tuple(grads)


class CircleLossFunction(torch.autograd.Function):
    """multi_circle_loss (cmu-mosei/run.py:342-351) on libmep_hip: returns the per-row loss."""

    @staticmethod
    def forward(ctx, y_pred, y_true):
        y_pred = y_pred.contiguous().float()
        B, NC = y_pred.shape
        lf = y_true.dtype.is_floating_point
        labels = y_true.contiguous().to(torch.float32 if lf else torch.int64)
        row = torch.empty(B, dtype=torch.float32, device=y_pred.device)
        dunit = torch.empty_like(y_pred)
        _lib.call('mep_circle_loss_fwd', ctypes.c_void_p(y_pred.data_ptr()), ctypes.c_void_p(labels.data_ptr()),
                  int(lf), B, NC, ctypes.c_void_p(row.data_ptr()), ctypes.c_void_p(dunit.data_ptr()))
        ctx.save_for_backward(dunit)
        return row

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad_rows):
        (dunit,) = ctx.saved_tensors
        B, NC = dunit.shape
        g = grad_rows.contiguous().float()
        out = torch.empty_like(dunit)
        _lib.call('mep_circle_loss_bwd', ctypes.c_void_p(dunit.data_ptr()), ctypes.c_void_p(g.data_ptr()), B, NC,
                  ctypes.c_void_p(out.data_ptr()))
        return out, None
