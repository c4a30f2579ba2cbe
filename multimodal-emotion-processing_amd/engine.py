"""Fused training-step engine: forward + loss + backward + [gradient all-reduce] + clip + AdamW
as a fixed launch sequence, captured once per input shape into a hipGraph and replayed.

Data parallelism (one process per GPU, torch.distributed backend "nccl" = RCCL over xGMI): each
rank runs the step on its own rows; the flat fp32 gradient buffer (2.35 MB for Concat_Trans)
is all-reduced (SUM) between the backward and the optimizer, and the optimizer clips
after the reduce, so every rank applies the identical update of the global-batch mean (1-GPU
large-batch semantics).  Two scalings give that mean:
  * global_rows given (a sharded batch, mep_amd.dp): the rank's loss is scaled by 1/B_global in
    the head kernel and the optimizer sees the plain SUM -- exact for unequal or empty shares;
  * global_rows None (every rank holds an equal share, e.g. bench.py): the local mean 1/B and
    grad_scale 1/world in the optimizer.
Ren-MME R-Drop pairs are whole units of a shard (mep_amd.dp), so they never straddle ranks.
With the nccl (= RCCL) backend the SUM is captured inside the step's hipGraph between the
backward and the optimizer (one graph launch per step), in two buckets of the flat buffer
(FlatParams.split): bucket A -- block weights, block LayerNorms and the fusion head, 86 % of the
gradient, complete after the last epilogue backward -- is all-reduced on a side stream while the
last attention backward, the per-modality sums and the unify weight gradients run; bucket B after
them.  With gloo (CPU tests) the SUM is a host call between two graph replays.
"""
import ctypes
import warnings

import torch
import torch.distributed as dist

from . import _lib


class TrainEngine:
    def __init__(self, model, optimizer, clip=1.0, rdrop=False, graph=True, process_group=None,
                 collective=None, capture_allreduce=None, fold_norm=None):
        """collective: run the flat-gradient all-reduce (default: when world > 1; True forces it
        at world 1, e.g. to exercise the RCCL path on one GPU).  capture_allreduce: capture the
        all-reduce inside the step's hipGraph between the backward and the optimizer (default:
        with the nccl = RCCL backend; gloo collectives are host calls and are never captured).
        fold_norm: single process, run the clip's norm pass inside the backward's reduction launch
        (default: on unless MEP_NORM_FOLD=0; its norm sums in another order than the optimizer's
        own pass, so runs compared bit for bit with a collective engine turn it off)."""
        self.model = model
        self.opt = optimizer
        self.clip = clip
        self.rdrop = rdrop
        self.graph = graph
        self.pg = process_group
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if dist_on else 1
        self.collective = (self.world > 1) if collective is None else (bool(collective) and dist_on)
        backend = dist.get_backend(process_group) if dist_on else None
        if capture_allreduce is None:
            env = _lib.switch('MEP_CAPTURE_ALLREDUCE', None)
            capture_allreduce = (env != '0') if env is not None else backend == 'nccl'
        self.capture_allreduce = bool(capture_allreduce) and self.collective and backend == 'nccl'
        # RCCL: bucket A of the flat gradient (FlatParams.split) is all-reduced on a side stream
        # while the rest of the backward runs (plans with backward_bucketed)
        env = _lib.switch('MEP_DP_OVERLAP', None)
        self.overlap = self.collective and backend == 'nccl' and (env != '0' if env is not None else True)
        self._side = None
        self._graphs = {}
        self.fold_norm = (_lib.switch('MEP_NORM_FOLD', '1') != '0') if fold_norm is None else bool(fold_norm)
        self._initial_broadcast = self.world > 1

    def _runner(self, device):
        return self.model.mep_runner(device)

    def plan(self, B, T, device):
        return self._runner(device).plan(B, T)

    # ---------------------------------------------------------------- step bodies
    def _fwd_bwd(self, plan):
        if plan._drop > 0.0:
            plan.advance_seed()
        plan.forward(grad=True, rdrop=self.rdrop)
        plan.backward()

    def _fwd_bwd_allreduce(self, plan, runner):
        """forward + backward + the gradient all-reduce; with overlap the first bucket's SUM runs
        on a side stream behind the last attention backward and the unify weight gradients"""
        if not (self.overlap and hasattr(plan, 'backward_bucketed')):
            self._fwd_bwd(plan)
            self._allreduce(runner)
            return
        flat = runner.flat
        a_end, n = flat.split, flat.n_grad
        if self._side is None:
            self._side = torch.cuda.Stream(device=flat.buf.device)
        side = self._side
        main = torch.cuda.current_stream()

        def bucket_a_done():
            side.wait_stream(main)
            with torch.cuda.stream(side):
                if a_end > 0:
                    dist.all_reduce(flat.grad[:a_end], op=dist.ReduceOp.SUM, group=self.pg)
        if plan._drop > 0.0:
            plan.advance_seed()
        plan.forward(grad=True, rdrop=self.rdrop)
        plan.backward_bucketed(bucket_a_done)
        if n > a_end:
            dist.all_reduce(flat.grad[a_end:n], op=dist.ReduceOp.SUM, group=self.pg)
        main.wait_stream(side)

    _n_ext = 0

    def _opt(self):
        if self._n_ext:
            self.opt.fused_step(n_ext=self._n_ext)
        else:
            self.opt.fused_step()

    def _norm_fold(self, plan):
        """Single process: the clip's gradient-norm pass runs inside the backward's reduction
        launch (mep_reduce_grads writes the norm partials and the step scalars into the optimizer
        workspace; one launch fewer per step).  With a gradient all-reduce the norm must follow
        the SUM, so the optimizer keeps its own norm pass."""
        fold = (self.fold_norm and not self.collective and hasattr(plan, 'reduce_grid')
                and hasattr(self.opt, 'norm_fold_ptrs'))
        n = plan.reduce_grid() if fold else 0
        fold = fold and 0 < n <= self.opt.MAX_EXT
        plan.norm_fold = self.opt.norm_fold_ptrs() if fold else None
        self._n_ext = n if fold else 0

    def _sync_params(self, runner):
        """Rank 0's parameters (and optimizer moments, all zero at start) to every rank."""
        if self._initial_broadcast:
            dist.broadcast(runner.flat.buf, 0, group=self.pg)
            self._initial_broadcast = False

    def step_plan(self, plan, global_rows=None, row0=0):
        """Run one training step on the data already in ``plan``'s input buffers; returns the loss
        as a device tensor (the local-batch mean, or with ``global_rows`` this rank's share of
        the global-batch mean).  row0: global index of the share's first row (dropout masks)."""
        runner = self._runner(plan.device)
        sharded = self.world > 1 and global_rows is not None
        self.opt._bind()
        self.opt._sync_hyper(self.clip, 1.0 if sharded else 1.0 / self.world)
        plan.set_dropout(runner.drop_p())
        # loss scale and dropout row offset are device-resident: one graph per plan serves every
        # share size (the head kernel reads them at replay)
        plan.set_global_rows(global_rows if sharded else None)
        if plan._drop > 0.0:
            plan.set_row0(row0 if sharded else 0)
        self._sync_params(runner)
        self._norm_fold(plan)
        key = id(plan)
        g = self._graphs.get(key)
        if not self.graph:
            self._fwd_bwd_allreduce(plan, runner)
            self._opt()
            return plan.loss
        if g is None:
            # first step eagerly (loads every kernel), then capture for the next ones
            self._fwd_bwd_allreduce(plan, runner)
            self._opt()
            torch.cuda.synchronize()
            split = self.collective and not self.capture_allreduce
            ga = None
            if not split:
                try:
                    ga = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(ga):
                        # RCCL all-reduce captured between the backward and the optimizer (its
                        # first bucket overlapping the end of the backward): one graph launch
                        self._fwd_bwd_allreduce(plan, runner)
                        self._opt()
                except RuntimeError as e:
                    if not self.collective:
                        raise
                    # a collective library that refuses capture: keep it outside the graph
                    warnings.warn('mep_amd: all-reduce capture failed (%s); running it between two '
                                  'graph replays' % (str(e).splitlines()[0] if str(e) else type(e).__name__))
                    torch.cuda.synchronize()
                    self.capture_allreduce, split, ga = False, True, None
            if split:
                ga = torch.cuda.CUDAGraph()
                with torch.cuda.graph(ga):
                    self._fwd_bwd(plan)
            gb = None
            if split:                 # gloo: host-side collective between two graph replays
                gb = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gb):
                    self._opt()
            self._graphs[key] = (ga, gb)
            return plan.loss
        ga, gb = g
        ga.replay()
        if gb is not None:
            self._allreduce(runner)
            gb.replay()
        return plan.loss

    def _allreduce(self, runner):
        if self.collective:
            dist.all_reduce(runner.flat.grad, op=dist.ReduceOp.SUM, group=self.pg)

    def step(self, *batch, global_rows=None, row0=0):
        """Reference-shaped batch in, loss out: the runner copies the batch into the resident
        buffers of the plan for its shape (cmu-mosei / Ren-MME: l, v, a, l_mask, v_mask, a_mask,
        labels; realformer: ... , labels, utterance mask)."""
        first = batch[0][0] if isinstance(batch[0], (tuple, list)) else batch[0]
        plan = self._runner(first.device).stage(*batch)
        return self.step_plan(plan, global_rows, row0)

    def step_empty(self, device):
        """A rank whose share of the (ragged, last) global batch is empty: zero gradient into the
        all-reduce, then the same optimizer step as every other rank.  The model's dropout seed
        advances as in a real step, so the ranks' seed streams stay equal."""
        runner = self._runner(torch.device(device))
        self.opt._bind()
        self.opt._sync_hyper(self.clip, 1.0)
        if runner.drop_p() > 0.0 and getattr(runner, 'seed_state', None) is not None:
            _lib.call('mep_seed_advance', ctypes.c_void_p(runner.seed_state.data_ptr()))
        self._sync_params(runner)
        runner.flat.grad.zero_()
        self._allreduce(runner)          # eager: an empty share is rare (the ragged last batch)
        self._n_ext = 0                  # no reduction ran: the optimizer's own norm pass
        self._opt()
        return torch.zeros(1, device=runner.flat.buf.device)


def engine_for(model, optimizer, **kw):
    """The TrainEngine of (model, optimizer, options), kept on the optimizer so the graphs it
    captured (one per batch shape) are replayed across epochs instead of re-captured by every
    train() call."""
    key = (id(model),) + tuple(sorted(kw.items()))
    cache = optimizer.__dict__.setdefault('_mep_engines', {})
    eng = cache.get(key)
    if eng is None or eng.model is not model:
        eng = cache[key] = TrainEngine(model, optimizer, **kw)
    return eng


class LossSum:
    """``epoch_loss += float(loss.item())`` of the reference train/valid loops without a host sync
    per batch: each fp32 loss is widened and added in float64 on the device, in batch order --
    the same IEEE double additions Python performs on the host, so the epoch value is identical,
    while the host runs ahead to stage the next batch."""

    def __init__(self):
        self.t = None

    def add(self, loss):
        l = loss.detach().reshape(()).double()
        if self.t is None:
            self.t = torch.zeros((), dtype=torch.float64, device=l.device)
        self.t.add_(l)

    def value(self):
        return float(self.t.item()) if self.t is not None else 0.0
