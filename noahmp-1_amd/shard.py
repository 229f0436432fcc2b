"""Column sharding across ranks (one process per GPU) and the output-step
diagnostics gather -- the path's only collective.

Columns are independent (no halo), so rank r owns a contiguous block of the
global column set; the diagnostics SoA of every rank (NDIAG_OUT x n_local) is
all-gathered at output steps into (world x NDIAG_OUT x n_local).  On "nccl"
(= RCCL on ROCm) this is one all_gather_into_tensor over xGMI; on "gloo" (CPU
tests) the list form.  When only one rank consumes the output (the offline
writer: rank 0 writes LDASOUT), ``dst`` turns it into a gather to that rank:
every sender pushes its block point-to-point straight to ``dst`` over its own
xGMI link instead of relaying through a ring, so total link traffic falls by
the world size and the root's N-1 incoming links run in parallel (SURVEY.md 8e,
"gather to root").
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
                async_op: bool = False, dst: int | None = None):
    """All-gather a (nfield, n_local) diagnostics block from every rank into
    out = (world * nfield, n_local) (rank-major).  Shards must be equal-sized.

    With ``dst`` (a global rank) only that rank receives: it gets ``out`` as
    above, every other rank gets None (its ``out`` argument is ignored)."""
    world = dist.get_world_size(group)
    if dst is not None and dist.get_rank() != dst:
        work = dist.gather(local.contiguous(), None, dst=dst, group=group, async_op=async_op)
        return (None, work) if async_op else None
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
    if out.shape[0] != world * local.shape[0] or out.shape[1:] != local.shape[1:]:
        raise ValueError(f"gather_diag: out {tuple(out.shape)} does not hold {world} blocks "
                         f"of {tuple(local.shape)}")
    if dst is not None:
        parts = list(out.view(world, *local.shape).unbind(0))
        work = dist.gather(local.contiguous(), parts, dst=dst, group=group, async_op=async_op)
    elif dist.get_backend(group) == "gloo":
        parts = list(out.view(world, *local.shape).unbind(0))
        work = dist.all_gather(parts, local.contiguous(), group=group, async_op=async_op)
    else:
        work = dist.all_gather_into_tensor(out, local.contiguous(), group=group, async_op=async_op)
    return (out, work) if async_op else out
