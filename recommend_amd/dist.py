"""Data-parallel gradient exchange over torch.distributed (RCCL over xGMI on MI355X; gloo in the
CPU tests).  The reference has no distribution code; the paper trains data-parallel with an
all-reduce (complete_translation.md:190).

* dense: the flat gradient buffer is all-reduced (one contiguous buffer -> no packing copies), then
  averaged (each rank's loss is a mean over its local batch).  In training the exchange overlaps the
  backward pass: every block's bank range (and the heads') is all-reduced on a communication stream
  as soon as it is final (OneTransOptimizer.begin_backward); the tokenizer's range, final last,
  goes in step().
* sparse (replicated tables): every rank all-gathers the (key, gradient-row) pairs of all
  ranks, scaled by 1/world, so each rank applies the identical de-duplicated Adagrad update.
"""

from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist

BUCKET_ELEMS = 8 * 1024 * 1024      # 32 MiB of fp32 per all-reduce


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def allreduce_dense(flat_grad: torch.Tensor, bucket_elems: int = BUCKET_ELEMS, scale: bool = True) -> None:
    """In-place mean (``scale``) or sum over ranks of a flat fp32 gradient buffer, bucketed."""
    w = world()
    if w == 1:
        return
    n = flat_grad.numel()
    works = []
    for s in range(0, n, bucket_elems):
        works.append(dist.all_reduce(flat_grad[s:s + bucket_elems], op=dist.ReduceOp.SUM, async_op=True))
    for wk in works:
        wk.wait()
    if scale:
        flat_grad.mul_(1.0 / w)


def allreduce_sum_async(t: torch.Tensor):
    """Asynchronous in-place sum over ranks (the caller's current stream orders it; wait() on the
    returned work makes the waiting stream depend on it)."""
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)


def allgather_sparse(keys: torch.Tensor, grads: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Concatenate every rank's (keys [n], grads [n, E]) in rank order; grads scaled by 1/world.
    All ranks contribute the same n (equal local batch shapes)."""
    w = world()
    if w == 1:
        return keys, grads
    ks = [torch.empty_like(keys) for _ in range(w)]
    gs = [torch.empty_like(grads) for _ in range(w)]
    dist.all_gather(ks, keys.contiguous())
    dist.all_gather(gs, grads.contiguous())
    return torch.cat(ks), torch.cat(gs).mul_(1.0 / w)
