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


def rank_local_params(module: torch.nn.Module) -> set:
    """ids of the rank-local parameters of `module` and its children: the per-sample betas
    (main_lena.py:35-36) of every submodule that is a batch shard (its `batch_shard` set by the
    batch_shard= constructor keyword or shard_batch_), found from the module structure itself --
    so a deep copy, or parameters re-registered by later code, are still recognised."""
    ids = set()
    for mod in module.modules():
        if getattr(mod, "batch_shard", None) is not None and hasattr(mod, "_elem_param_lists"):
            for pl in mod._elem_param_lists():
                ids.update(id(p) for p in pl)
    return ids


def allreduce_grads(module: torch.nn.Module, group: Optional[dist.ProcessGroup] = None,
                    average: bool = False) -> None:
    """Data-parallel training over batch shards: ONE all-reduce of every parameter gradient,
    flattened into a single bucket (the whole D-LADMM parameter set is a few MB: K weights of
    n x m plus per-layer scalars), then scattered back.  With `training_loss(..., batch=B_global)`
    each rank's gradient is its shard's share of the global-batch objective, so SUM (the default)
    gives the full-batch gradient; `average=True` divides by the world size instead (losses
    normalised by the local batch).
    Rank-local parameters -- V1's per-sample betas of a module that is a batch shard
    (main_lena.py:35-36: one column per sample; rank_local_params) -- are not in the bucket: their
    gradient is already complete on the rank that holds those columns."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    local = rank_local_params(module)
    ps = [p for p in module.parameters() if p.grad is not None and id(p) not in local]
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


def gather_state_dict(module: torch.nn.Module, group: Optional[dist.ProcessGroup] = None):
    """The reference-layout state_dict of a batch-sharded module (`shard_batch_`), for saving
    (main_lena.py:243 `torch.save(model.state_dict(), ...)`): every rank-local per-sample beta
    is all-gathered along its columns back to (m, batch_size); replicated entries are this
    rank's (equal on every rank).  A collective: every rank calls it.  Unsharded modules (or one
    rank) return their own state_dict."""
    sd = module.state_dict()
    shard = getattr(module, "batch_shard", None)
    if shard is None:
        return sd
    c0, c1, B = shard
    up = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if up else 1
    rank = dist.get_rank(group) if up else 0
    if tuple(getattr(module, "world", (rank, world))) != (rank, world):
        raise RuntimeError(f"dladmm: the module is shard {module.world} (rank, world) but the "
                           f"process group is rank {rank} of {world}")
    local = {f"{nm}.{k}" for nm in module._elem_names() for k in range(module.layers)}
    if world == 1:
        if c1 - c0 != B:
            raise RuntimeError("dladmm: a batch shard needs its process group to gather")
        return sd
    spans = [shard_columns(B, r, world) for r in range(world)]
    wmax = max(b - a for a, b in spans)
    for key in sorted(local):
        v = sd[key]
        pad = torch.zeros((v.shape[0], wmax), dtype=v.dtype, device=v.device)
        pad[:, :v.shape[1]] = v
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        sd[key] = torch.cat([p[:, :b - a] for p, (a, b) in zip(parts, spans)], 1)
    return sd
