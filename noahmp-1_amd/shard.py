"""Column sharding across ranks (one process per GPU) and the output-step
diagnostics gather -- the path's only collective.

Columns are independent (no halo), so rank r owns a contiguous block of the
global column set (`shard_range`; the first ncol % world ranks hold one
column more).  At output steps the diagnostics SoA of every rank (nfield x
n_local) is gathered.  On "nccl" (= RCCL on ROCm) this is one collective over
xGMI; on "gloo" (CPU tests) the list form.  When only one rank consumes the
output (the offline writer: rank 0 writes LDASOUT), ``dst`` turns it into a
gather to that rank: every sender pushes its block point-to-point straight to
``dst`` over its own xGMI link instead of relaying through a ring, so total
link traffic falls by the world size and the root's N-1 incoming links run in
parallel ("gather to root").

Ragged shards: a collective moves equal-sized blocks, so every rank's block
travels in a slot of nfield * max(n_local) elements.  A rank's (nfield,
n_local) diagnostics are the contiguous prefix of its slot (rows n_local
apart, the layout the engine writes), and `DiagGather.assemble` trims each
slot back to its rank's columns.
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
    """All-gather an equal-sized block (any shape) from every rank into
    out = (world * local.shape[0], *local.shape[1:]) (rank-major).

    With ``dst`` (a global rank) only that rank receives: it gets ``out`` as
    above, every other rank gets None (its ``out`` argument is ignored).
    Ragged shards go through `DiagGather`, which pads them into equal slots."""
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


class DiagGather:
    """Output-step diagnostics gather with ragged shards and `nbuf` buffers.

    Each buffer is one flat slot per rank on the receiving rank(s) (dst, or
    every rank for dst=None) and a single slot on a pure sender.  `local(b)`
    is the (nfield, n_local) block this rank's engine writes for buffer b; on
    a receiver it IS this rank's slot of the gather buffer, so the collective
    copies nothing locally.  `start(b)` issues the asynchronous collective on
    `comm` (a side stream on GPUs) once `producers` are done, `release(b)`
    makes streams wait until buffer b may be overwritten, `assemble(b)` is the
    receiver's (nfield, ncol_total) result in global column order.

    On a gloo group with CUDA buffers the slot is staged through host memory
    (gloo moves host tensors); the staging is synchronous."""

    def __init__(self, nfield: int, ncol_total: int, dtype, device, dst: int | None = 0,
                 nbuf: int = 2, group=None, comm: torch.cuda.Stream | None = None,
                 force_collective: bool = False, wire_dtype=None):
        """force_collective: issue the collective even on a single rank (where
        nothing needs to move), so the RCCL code path of a multi-GPU run can
        be executed and checked on one GPU (tests/probe_rccl_gather.py).
        wire_dtype: the gathered values' type when it differs from the
        engine's `dtype` (e.g. fp32 fluxes of an fp64 run, half the link
        bytes): the engine writes `local(b)` in dtype, `start` converts it
        into the wire buffer on the issuing stream, `assemble` returns
        wire_dtype."""
        self.force_collective = bool(force_collective)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dst = dst
        self.nfield = nfield
        self.counts = [shard_range(ncol_total, r, self.world)[1] for r in range(self.world)]
        self.n_local = self.counts[self.rank]
        self.slot = nfield * max(max(self.counts), 1)
        self.device = torch.device(device)
        self.receives = dst is None or self.rank == dst
        self.staged = dist.get_backend(group) == "gloo" and self.device.type == "cuda"
        nslot = self.world if self.receives else 1
        wire = dtype if wire_dtype is None else wire_dtype
        self.bufs = [torch.zeros(nslot * self.slot, dtype=wire, device=self.device)
                     for _ in range(nbuf)]
        # engine-precision blocks the engine writes when the wire type differs
        self.src = [torch.zeros((nfield, self.n_local), dtype=dtype, device=self.device)
                    for _ in range(nbuf)] if wire != dtype else None
        self.host = [torch.zeros(nslot * self.slot, dtype=wire) for _ in range(nbuf)] \
            if self.staged else None
        self.comm = comm
        self.pending = [None] * nbuf   # host-side work handles (CPU buffers)
        self.done = [None] * nbuf      # CUDA buffers: event after buffer b's last collective
        self.local_producers = [[] for _ in range(nbuf)]

    def _slot(self, buf: torch.Tensor, r: int) -> torch.Tensor:
        return buf[r * self.slot:(r + 1) * self.slot]

    def _own(self, b: int) -> torch.Tensor:
        own = self._slot(self.bufs[b], self.rank if self.receives else 0)
        return own[:self.nfield * self.n_local].view(self.nfield, self.n_local)

    def local(self, b: int) -> torch.Tensor:
        return self.src[b] if self.src is not None else self._own(b)

    def _convert(self, b: int):
        """(wire_dtype differs) the engine's block into the wire buffer, on the
        current stream."""
        if self.src is not None:
            self._own(b).copy_(self.src[b])

    def start(self, b: int, producers=()):
        """Issue the gather of buffer b after every stream in `producers` (e.g.
        the StreamShards range streams that wrote local(b)).  A single rank
        already holds its block in its slot: nothing moves, no collective runs
        (an in-place self-gather of 64 MB under RCCL cost 4 % of the N = 1
        bench, the collective's kernel taking CUs from the step)."""
        if self.world == 1 and not self.force_collective:
            self.local_producers[b] = list(producers)  # assemble() waits for them
            if self.src is not None:
                if self.device.type == "cuda":
                    for s in producers:
                        torch.cuda.current_stream(self.device).wait_stream(s)
                self._convert(b)
                self.local_producers[b] = []
            return
        bufs = self.host if self.staged else self.bufs
        if self.staged:
            for s in producers:
                torch.cuda.current_stream(self.device).wait_stream(s)
            self._convert(b)
            bufs[b].copy_(self.bufs[b])
            self._issue(b, bufs[b], async_op=False)
            if self.receives:
                self.bufs[b].copy_(bufs[b])
            return
        if self.comm is not None:
            for s in producers:
                self.comm.wait_stream(s)
            with torch.cuda.stream(self.comm):
                self._convert(b)
                self._issue(b, bufs[b], async_op=True)
                self._fence(b)
        else:
            if self.device.type == "cuda":
                for s in producers:
                    torch.cuda.current_stream(self.device).wait_stream(s)
            self._convert(b)
            self._issue(b, bufs[b], async_op=True)
            self._fence(b)

    def _fence(self, b: int):
        """CUDA buffers: the issuing stream waits for buffer b's collective (a
        device-side wait, the host does not block) and an event recorded after
        it becomes the buffer's fence.  It stays in place until the buffer's
        next collective, so every later writer (`release`, however many
        times) and reader (`assemble`) is ordered after the transfer -- none
        can consume the fence and leave another stream unordered."""
        if self.device.type != "cuda" or self.pending[b] is None:
            return
        self.pending[b].wait()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.done[b], self.pending[b] = ev, None

    def _issue(self, b: int, buf: torch.Tensor, async_op: bool):
        own = self._slot(buf, self.rank if self.receives else 0)
        if self.receives:
            parts = [self._slot(buf, r) for r in range(self.world)]
            if self.dst is not None:
                w = dist.gather(own, parts, dst=self.dst, group=self.group, async_op=async_op)
            elif dist.get_backend(self.group) == "gloo":
                w = dist.all_gather(parts, own, group=self.group, async_op=async_op)
            else:
                w = dist.all_gather_into_tensor(buf, own, group=self.group, async_op=async_op)
        else:
            w = dist.gather(own, None, dst=self.dst, group=self.group, async_op=async_op)
        self.pending[b] = w if async_op else None

    def release(self, b: int, streams=()):
        """Make `streams` (default: the current stream) wait until the collective
        that last used buffer b is done, so it can be written again."""
        if self.done[b] is not None:
            for s in (streams or [torch.cuda.current_stream(self.device)]):
                s.wait_event(self.done[b])
            return
        w = self.pending[b]
        if w is None:
            return
        w.wait()  # CPU buffers: blocks the host until the collective is done
        self.pending[b] = None

    def assemble(self, b: int) -> torch.Tensor | None:
        """Receiver: (nfield, ncol_total) diagnostics of buffer b in global
        column order (waits for its collective on the current stream); None on
        a pure sender."""
        self.release(b)
        if not self.receives:
            return None
        if self.device.type == "cuda":
            for st in self.local_producers[b]:
                torch.cuda.current_stream(self.device).wait_stream(st)
        self.local_producers[b] = []
        blocks = [self._slot(self.bufs[b], r)[:self.nfield * c].view(self.nfield, c)
                  for r, c in enumerate(self.counts)]
        return torch.cat(blocks, dim=1)

    def wait_all(self):
        for b in range(len(self.bufs)):
            self.release(b)


class OutputSchedule:
    """The output-step loop shared by bench.py and the offline driver.

    Step k writes diagnostics when (k + 1) % out_every == 0, into buffer
    (k // out_every) % nbuf, so output step j+1 fills the other buffer while
    output step j's gather may still be in flight.  `diag_for(k)` returns the
    block step k writes (None on plain steps), after making `streams` wait for
    the collective that last used that buffer; `finish(k, producers)` starts the
    gather of an output step once `producers` (the streams that wrote it) are
    done.  Without a DiagGather (single rank) `bufs` are plain local blocks."""

    def __init__(self, out_every: int, gather: DiagGather | None = None, bufs=None,
                 streams=()):
        assert out_every >= 1 and (gather is not None or bufs)
        self.out_every, self.gather, self.bufs = out_every, gather, bufs
        self.streams = list(streams)
        self.nbuf = len(gather.bufs) if gather is not None else len(bufs)

    def is_output(self, k: int) -> bool:
        return (k + 1) % self.out_every == 0

    def buffer(self, k: int) -> int:
        return (k // self.out_every) % self.nbuf

    def diag_for(self, k: int):
        if not self.is_output(k):
            return None
        b = self.buffer(k)
        if self.gather is None:
            return self.bufs[b]
        self.gather.release(b, self.streams)
        return self.gather.local(b)

    def finish(self, k: int, producers=()):
        if self.is_output(k) and self.gather is not None:
            self.gather.start(self.buffer(k), producers)
