"""Batch-sharded data parallelism for the fused forward.

Columns of X are independent samples, so the only data-path partitioning is a contiguous column
shard per rank (A, W_k and the per-layer parameters are replicated); the only exchange is ONE
all-reduce of the [K, 2] per-layer objective sums (RCCL over xGMI with the "nccl" backend, gloo on
CPU).  There is no output gather: every rank keeps its shard of Z/E/L/T.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_columns(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, stop) column range of `rank` (sizes differ by at most one)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} not in [0, {world})")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def global_objectives(local_sums: torch.Tensor, alpha: float, total_batch: int,
                      group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Per-layer objective of the whole (sharded) batch from each rank's [K, 2] sums
    (sum|Z_k|, fit_k): one all-reduce(SUM), then (alpha*sum|Z| + fit) / B_total, i.e. the
    reference's alpha*sum(|Z|,0).mean() + sum(|X-AZ|,0).mean() (main_syn_l1l1_scalar.py:290-294)
    over all ranks' columns."""
    s = local_sums
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        s = s.clone()  # the caller's sums stay its shard's
        dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    # (alpha * sum|Z| + fit) / B in two small kernels
    return torch.add(s[:, 1], s[:, 0], alpha=alpha).div_(total_batch)


def allreduce_grads(module: torch.nn.Module, group: Optional[dist.ProcessGroup] = None,
                    average: bool = False) -> None:
    """Data-parallel training over batch shards: ONE all-reduce of every parameter gradient,
    flattened into a single bucket (the whole D-LADMM parameter set is a few MB: K weights of
    n x m plus per-layer scalars), then scattered back.  With `training_loss(..., batch=B_global)`
    each rank's gradient is its shard's share of the global-batch objective, so SUM (the default)
    gives the full-batch gradient; `average=True` divides by the world size instead (losses
    normalised by the local batch)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    ps = [p for p in module.parameters() if p.grad is not None]
    if not ps:
        return
    flat = torch.cat([p.grad.reshape(-1) for p in ps])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    if average:
        flat /= dist.get_world_size(group)
    o = 0
    for p in ps:
        n = p.grad.numel()
        p.grad.copy_(flat[o:o + n].view_as(p.grad))
        o += n
