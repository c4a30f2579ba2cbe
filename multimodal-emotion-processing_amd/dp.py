"""Data-parallel epoch plumbing: one process per GPU, torch.distributed backend
"nccl" (= RCCL over xGMI on ROCm; "gloo" in the CPU tests).

The reference trains on one device (cmu-mosei/run.py:18) with ``loss.mean()`` over the rows of a
batch.  Here a *global* batch is split over the ranks and every rank runs the fused step on its
share with the loss scaled by 1/B_global (the head kernel's ``loss_scale``, and the R-Drop KL's
batchmean divisor set to the global pair count), so the SUM all-reduce of the flat gradient is
exactly the gradient of the global-batch mean -- also for the ragged last batch, where the ranks'
shares differ or are empty.  The epoch losses that drive ReduceLROnPlateau and early stopping
(cmu-mosei/run.py:371,389,409) are summed over ranks once per epoch, so every rank takes the same
learning-rate and checkpoint decisions; only rank 0 writes files.

Sharding keeps the reference's row order: the batch order comes from ``random.shuffle`` on rank 0
(broadcast to the others), global batch k holds units [k * B * world, (k + 1) * B * world) of
that order, and rank r takes units [r * B, (r + 1) * B) of it.  A unit is a (previous, current)
utterance pair for cmu-mosei, a group of P utterances for realformer and a duplicated sample pair
(rows 2i, 2i + 1) for Ren-MME, whose R-Drop KL compares the two rows (Ren-MME/run.py:143-146,
332-333) -- so a pair never straddles ranks.
"""
import random

import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def shared_shuffle(name_list):
    """``random.shuffle(name_list)`` in place (the reference's call) with rank 0's order on every
    rank."""
    random.shuffle(name_list)
    if world() > 1:
        obj = [list(name_list)]
        dist.broadcast_object_list(obj, src=0)
        name_list[:] = obj[0]
    return name_list


def rank_range(n_units, per_rank, r=None):
    """Units [lo, hi) of rank r in a global batch of n_units units, per_rank units per rank."""
    r = rank() if r is None else r
    return min(n_units, r * per_rank), min(n_units, (r + 1) * per_rank)


class HostShard(list):
    """This rank's rows of a host-layout batch (a list of row tuples, as the reference's
    data_loader yields them); ``global_rows`` = rows of the whole global batch, ``row0`` = the
    global index of this share's first row (the dropout masks of row b are those of global row
    row0 + b, so the ranks together draw exactly the full batch's masks)."""

    def __init__(self, rows, global_rows, row0=0):
        super().__init__(rows)
        self.global_rows = int(global_rows)
        self.row0 = int(row0)


def shard_batches(iterator, unit=1, per_rank=None):
    """Wrap a reference-style data_loader generator whose items are GLOBAL batches: yields this
    rank's HostShard of each (contiguous units of ``unit`` rows; unit=2 for Ren-MME pairs).
    per_rank: units per rank (default: an even split, ceil(units / world))."""
    w, r = world(), rank()
    for batch in iterator:
        n = len(batch)
        if n % unit:
            raise ValueError('shard_batches: %d rows is not a whole number of %d-row units' % (n, unit))
        units = n // unit
        per = per_rank if per_rank is not None else -(-units // w)
        lo, hi = rank_range(units, per, r)
        yield HostShard(batch[lo * unit:hi * unit], n, lo * unit)


def allreduce_sum(values, device=None):
    """Sum of a few host floats over the ranks (float64), one collective."""
    if world() == 1:
        return [float(v) for v in values]
    dev = device if device is not None and dist.get_backend() != 'gloo' else torch.device('cpu')
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu()]


def global_rows_of(batch):
    """``global_rows`` of a sharded batch, or None (an unsharded, rank-local batch)."""
    return getattr(batch, 'global_rows', None)


def row0_of(batch):
    """Global index of a sharded batch's first row (0 for an unsharded batch)."""
    return int(getattr(batch, 'row0', 0) or 0)


def epoch_mean(local_sum, count, sharded, device=None):
    """Epoch value of the reference's ``epoch_loss / count`` (cmu-mosei/run.py:371-372) under data
    parallelism: sharded batches carry each rank's share of the global-batch loss (summed over
    ranks); unsharded ones are rank-local batch means of equal shares (averaged over ranks)."""
    if world() == 1:
        return local_sum / count if count else 0.0
    (total,) = allreduce_sum([local_sum], device)
    if not sharded:
        total /= world()
    return total / count if count else 0.0
