"""Column sharding across ranks (one process per GPU) and the output-step
diagnostics gather -- the path's only collective.

Columns are independent (no halo), so rank r owns a contiguous block of the
global column set; the diagnostics SoA of every rank (NDIAG_OUT x n_local) is
all-gathered at output steps into (world x NDIAG_OUT x n_local).  On "nccl"
(= RCCL on ROCm) this is one all_gather_into_tensor over xGMI; on "gloo" (CPU
tests) the list form.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(ncol_total: int, rank: int, world: int) -> tuple[int, int]:
    """(start, count) of rank's contiguous block; remainders go to the low ranks."""
    assert 0 <= rank < world and ncol_total >= 0
    base, rem = divmod(ncol_total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def gather_diag(local: torch.Tensor, out: torch.Tensor | None = None, group=None,
                async_op: bool = False):
    """All-gather a (nfield, n_local) diagnostics block from every rank into
    out = (world * nfield, n_local) (rank-major).  Shards must be equal-sized."""
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
    if dist.get_backend(group) == "gloo":
        parts = list(out.view(world, *local.shape).unbind(0))
        work = dist.all_gather(parts, local.contiguous(), group=group, async_op=async_op)
    else:
        work = dist.all_gather_into_tensor(out, local.contiguous(), group=group, async_op=async_op)
    return (out, work) if async_op else out
