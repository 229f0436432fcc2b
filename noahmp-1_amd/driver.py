"""Offline driver: the time loop behind run/main.py.

The reference's driver parses the namelist and stops (run/main.py:12-14;
offline/noahmp_config.py has no time loop, forcing reader or writer, SURVEY
8f).  `OfflineDriver` is that missing loop around the engine:

* steps begdatetime -> enddatetime by `timestep` (Config), calling
  `Engine.step` for every column each step; JULIAN / YEARLEN / COSZ are
  computed per step at the step's start time (timeman.py);
* forcing comes from a provider `forcing(step, t) -> (12, n)` array; the
  reference's LDASIN files are not in the repository, so `SyntheticForcing`
  (the seeded diurnal generator the tests and bench use) is the default;
  `forcing="device"` generates the synthetic forcing on the GPU instead
  (`DeviceSyntheticForcing`, nmp_forcing_synth);
* output steps (Config.output_frequency) write the 16 surface fluxes as
  ``<outdir>/<YYYYMMDDHH>.LDASOUT_DOMAIN1`` (netCDF-3 on the grid, ncio.py)
  when the columns come from a grid, else ``<outdir>/<YYYYMMDDHH>.LDASOUT.npz``;
* restart steps (Config.restart_frequency, calendar months allowed) write the
  complete SoA state (``RESTART.<YYYYMMDDHH>_DOMAIN1.nc`` on a grid, else
  ``.npz``), which `load_restart` reads back -- the state SoA *is* the restart
  (SURVEY 8f item 2);
* `OfflineDriver.from_files` builds the run from the namelist's files: the
  static file (grid, types), the initialization file (state) and the LDASIN
  directory (forcing), all netCDF-3 (ncio.py).

Multi-rank: each rank drives its own column shard (shard.shard_range of the
land points; `from_files` reads only its slice); at output steps the
diagnostics are gathered to rank 0 (shard.DiagGather, dst=0, ragged shards
allowed), which writes them for the whole grid.

Forcing reaches the GPU through `ForcingUpload`: pinned, double-buffered
host buffers copied on a copy stream, so the host builds step t+1's forcing
while the GPU steps t.  From LDASIN files (cosz="device", ingest=True, the
defaults) a file's bytes go up as stored, once per input interval
(ncio.LdasinForcing.grid_raw, read ahead on a thread), and the engine forms
the block in its column order (nmp_ldasin_ingest) on the upload stream,
beside the steps of the previous file; the block stays resident while each
range forms the 12 forcing fields, COSZ included, on its own stream right
before its launch (nmp_forcing_from_ldasin_geo), waiting only on that
block's event.  ingest=False builds the block on the host
(ncio.LdasinForcing.block); cosz="host" uploads the variables plus the
host's COSZ every step (ncio.LdasinForcing.raw, nmp_forcing_from_ldasin);
the 12-field host form (48 B per column, 96 in fp64) remains for providers
that supply all of them.  A single rank's output is laid on the file's grids
(nmp_ldasout_grid) and copied on a stream of its own and written by writer
threads (ncio.write_ldasout_grids).

`phase_s` accumulates the host time of the loop's parts (file headers,
forcing, launch enqueue, output hand-off, the whole iteration), for the
offline-driver timing (tools/offline_timing.py).
"""
from __future__ import annotations

import datetime
import os
import time
from collections import defaultdict

import numpy as np
import torch
import torch.distributed as dist

from . import cases, layout as L, ncio, shard, timeman
from .config import Config
from .engine import ColumnState, Engine, StreamShards
from .order import coherent_order
from .params import Params


class SyntheticForcing:
    """Seeded diurnal forcing for a ColumnSet (cases.forcing_step), per step."""

    def __init__(self, cols: cases.ColumnSet, seed: int = 0):
        self.cols, self.seed = cols, seed

    def __call__(self, step: int, t: datetime.datetime) -> np.ndarray:
        return cases.forcing_step(self.cols, timeman.julian(t), timeman.yearlen(t.year), step,
                                  seed=self.seed)


class ForcingUpload:
    """Pinned, double-buffered host->device forcing uploads on a copy stream.

    `put(f)` copies the (12, n) host array into pinned buffer b, enqueues its
    upload to device buffer b on the copy stream and returns that device
    buffer; the caller's launches wait on `stream`.  Buffer b is reused two
    puts later: the host side waits for b's previous upload to land, the copy
    stream for the launches that read it (`consumed_by`)."""

    def __init__(self, n: int, dtype, device, nbuf: int = 2, nfield: int = L.NFORCING):
        dev = torch.device(device)
        self.host = [torch.empty((nfield, n), dtype=dtype, pin_memory=True)
                     for _ in range(nbuf)]
        self.dev = [torch.empty((nfield, n), dtype=dtype, device=dev) for _ in range(nbuf)]
        self.stream = torch.cuda.Stream(dev)
        self.uploaded = [None] * nbuf
        self.consumed = [()] * nbuf
        self.count = 0

    def put(self, f: np.ndarray | None = None, fill=None, prefilled: bool = False) -> torch.Tensor:
        """Upload f, or whatever fill(host_array) writes into the pinned buffer
        (a provider filling it in place saves a host copy), or -- prefilled --
        what a completed prefetch() left there."""
        b = self.count % len(self.host)
        self.count += 1
        if prefilled:
            pass  # prefetch() waited for the buffer's previous upload and filled it
        else:
            if self.uploaded[b] is not None:
                self.uploaded[b].synchronize()  # pinned buffer b is free again
            if fill is not None:
                fill(self.host[b].numpy())
            else:
                self.host[b].numpy()[...] = f
        for e in self.consumed[b]:
            self.stream.wait_event(e)
        with torch.cuda.stream(self.stream):
            self.dev[b].copy_(self.host[b], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.uploaded[b], self.consumed[b] = ev, ()
        self._last = b
        return self.dev[b]

    def prefetch(self, fill, executor):
        """Fill the pinned buffer the next put() will use on `executor`, once
        its previous upload has landed; the caller then calls put(prefilled=
        True) after the returned future has completed without error."""
        b = self.count % len(self.host)
        ev, h = self.uploaded[b], self.host[b].numpy()

        def job():
            if ev is not None:
                ev.synchronize()
            fill(h)
        return executor.submit(job)

    @property
    def last_slot(self) -> int:
        """The buffer slot of the last put (its device buffer and whatever the
        caller keeps per slot are guarded by the same events)."""
        return self._last

    def consumed_by(self, streams, slot: int | None = None):
        """The last put's device buffer (or slot `slot`'s) is read by launches
        on `streams`."""
        evs = []
        for s in streams:
            e = torch.cuda.Event()
            e.record(s)
            evs.append(e)
        self.consumed[self._last if slot is None else slot] = tuple(evs)


class DeviceSyntheticForcing:
    """Synthetic forcing generated on the device each step (nmp_forcing_synth):
    no host generation, no upload -- the long-run path for synthetic cases
    (a year of hourly forcing for 1 M columns would be 0.4-0.8 TB from the
    host).  climate: (NCLIM, n) records of this rank's columns
    (cases.climate); first_col: their global index (stateless draws)."""
    on_device = True

    def __init__(self, climate: np.ndarray, seed: int = 0, first_col: int = 0):
        self.climate, self.seed, self.first_col = climate, seed, first_col


def _stamp(t: datetime.datetime) -> str:
    return t.strftime("%Y%m%d%H")


def _is_boundary(t: datetime.datetime, t0: datetime.datetime, every) -> bool:
    if every is None:
        return False
    if isinstance(every, str):  # 'Nmonth': calendar month boundaries at 00:00 of day 1
        n = int(every[:-5])
        months = (t.year - t0.year) * 12 + (t.month - t0.month)
        return t.day == 1 and t.hour == 0 and t.minute == 0 and t.second == 0 and months % n == 0 \
            and t != t0
    return (t - t0) % every == datetime.timedelta(0)


def _global_count(n: int, dev) -> int:
    """Sum of the ranks' column counts."""
    on_host = dist.get_backend() == "gloo"
    t = torch.tensor([n], dtype=torch.int64, device="cpu" if on_host else dev)
    dist.all_reduce(t)
    return int(t.item())


class OfflineDriver:
    def __init__(self, cfg: Config, cols: cases.ColumnSet, device: int = 0,
                 params: Params | None = None, forcing=None, precision: int = 4,
                 math: str = "ref", zsoil=cases.CASE_NML_ZSOIL, write: bool = True,
                 streams: int = 2, grid: ncio.Grid | None = None, ldasin_upload: bool = True,
                 cosz: str = "device", ingest: bool = True):
        """cols: this rank's columns (all of them on a single rank); under an
        initialised process group they must be the rank's shard_range block of
        the global column set.  ldasin_upload: with a provider that has
        `raw` (LDASIN files), upload the files' variables and form the forcing
        on the device (False: the 12-field host form, for comparison).
        cosz: with ldasin_upload, "device" forms COSZ on the device from the
        columns' geometry (the files' variables then go up once per input
        interval), "host" computes it on the host and uploads it every step.
        ingest: with cosz="device", upload each file's bytes as it stores them
        (its big-endian grids, ncio.LdasinForcing.grid_raw) and select, order
        and byte-swap this rank's columns on the device (nmp_ldasin_ingest)
        instead of on the host (ncio.LdasinForcing.block)."""
        if cosz not in ("device", "host"):
            raise ValueError(f"cosz must be 'device' or 'host', not {cosz!r}")
        self.cfg = cfg
        self.grid = grid
        self.engine = Engine(params or Params.builtin(), cfg.engine_options(), device, precision,
                             math)
        self.dtype = self.engine.dtype
        self.dev = torch.device("cuda", device)
        self.cs = ColumnState.from_host(cols, self.dev, self.dtype)
        # column ranges on their own streams: launch tails overlap (engine.StreamShards)
        self.ranges = StreamShards(self.engine, self.cs, streams)
        total, first = self.cs.ncol, 0
        if dist.is_initialized():
            total = _global_count(self.cs.ncol, self.dev)
            first = shard.shard_range(total, dist.get_rank(), dist.get_world_size())[0]
        if forcing == "device":
            # draws keyed by the global column index: the forcing of a column
            # does not depend on the world size
            forcing = DeviceSyntheticForcing(cases.climate(cols), seed=0, first_col=first)
        self.forcing = forcing or SyntheticForcing(cols)
        self.dev_forcing = None
        if getattr(self.forcing, "on_device", False):
            # two device buffers: step k writes buffer k % 2 on each range's
            # stream right before that range's launch (stream order: reuse safe)
            self.dev_forcing = (
                torch.as_tensor(self.forcing.climate, device=self.dev).to(self.dtype).contiguous(),
                torch.empty((2, L.NFORCING, self.cs.ncol), dtype=self.dtype, device=self.dev))
        self.zsoil = [float(z) for z in zsoil]
        self.dt = cfg.timestep.total_seconds()
        self.t = cfg.begdatetime
        self.step_index = 0
        self.write = write
        self.diag = torch.zeros((L.NDIAG_OUT, self.cs.ncol), dtype=self.dtype, device=self.dev)
        self.upload = ForcingUpload(self.cs.ncol, self.dtype, self.dev)
        self.raw_upload = None
        if ldasin_upload and hasattr(self.forcing, "raw") and self.dev_forcing is None:
            self.raw_upload = ForcingUpload(self.cs.ncol, torch.float32, self.dev,
                                            nfield=L.NLDASIN)
            self.raw_fbuf = torch.empty((2, L.NFORCING, self.cs.ncol), dtype=self.dtype,
                                        device=self.dev)
        self.geo, self._blocks = None, {}
        self._prefetch, self._prefetch_pool = None, None
        # single-rank output: grids and copies on a stream of their own, so the
        # next steps need not wait for them (only the next output step waits
        # for the diagnostics buffer to be read: _diag_free)
        self.out_stream, self._diag_free = None, None
        if self.raw_upload is not None and cosz == "device":
            self.geo = torch.as_tensor(self.forcing.geo(), device=self.dev).contiguous()
        self.ingest = None
        if self.geo is not None and ingest and hasattr(self.forcing, "grid_raw"):
            npts = self.forcing.grid.shape[0] * self.forcing.grid.shape[1]
            self.ingest = ForcingUpload(npts, torch.int32, self.dev, nfield=L.NLDASIN - 1)
            self.ingest_blk = torch.zeros((2, L.NLDASIN, self.cs.ncol), dtype=torch.float32,
                                          device=self.dev)
            self.point = torch.as_tensor(self.forcing.point(), device=self.dev)
        self.phase_s = defaultdict(float)
        self.gather = None
        if dist.is_initialized():
            self.gather = shard.DiagGather(L.NDIAG_OUT, total, self.dtype, self.dev, dst=0)
            if self.gather.n_local != self.cs.ncol:
                raise ValueError(f"rank {dist.get_rank()} holds {self.cs.ncol} columns, its "
                                 f"shard_range block of {total} has {self.gather.n_local}")
        self.n_out = 0
        self.written = []
        self._writer = None
        if write and cfg.output_interval is not None and (
                not dist.is_initialized() or dist.get_rank() == 0):
            # the output staging buffers up front: a page-locked allocation of
            # the whole set's fluxes costs tens of ms inside the time loop (the
            # file's grids in its byte order when the run has a grid)
            if grid is not None:
                self._writer_init((L.NDIAG_OUT, grid.shape[0] * grid.shape[1]),
                                  torch.int32 if self.dtype == torch.float32 else torch.int64)
            else:
                self._writer_init((L.NDIAG_OUT, total))
        self._out_point = None

    @classmethod
    def from_files(cls, cfg: Config, device: int = 0, params: Params | None = None,
                   init: str | None = None, order: str | None = "lon-snow-type",
                   host_threads: int | None = None, **kw) -> "OfflineDriver":
        """The run the namelist describes: static file (cfg.constfile), initial
        state (cfg.initfile, or `init`) and LDASIN forcing (cfg.indir every
        cfg.input_frequency), netCDF-3 files in the layouts of ncio.py.

        order: the land points are laid out in the engine in this coherent
        order (order.coherent_order; None = grid order).  The permutation is
        applied when columns are read from the files and undone when they are
        written, so files always hold the grid.
        host_threads: threads that build each step's forcing on the host
        (ncio.LdasinForcing; default NMP_HOST_THREADS, else 8)."""
        P = params or Params.builtin()
        grid, sf, si = ncio.read_static(cfg.constfile, P.as_dict(), cfg.begdatetime)
        st, isn, t0, step = ncio.read_state(init or cfg.initfile, grid)
        perm = np.arange(grid.n) if order is None else coherent_order(grid.lon_rad, si, isn,
                                                                      order, band_deg=4.0)
        idx = perm
        if dist.is_initialized():  # this rank's block of the (ordered) land points
            s0, cnt = shard.shard_range(grid.n, dist.get_rank(), dist.get_world_size())
            idx = perm[s0:s0 + cnt]
        cols = cases.ColumnSet(sf[:, idx], si[:, idx], st[:, idx], isn[idx], grid.lon_rad[idx],
                               *([None] * 6))
        forcing = ncio.LdasinForcing(cfg.indir, grid, cfg.begdatetime, cfg.input_interval,
                                     cols=idx, threads=host_threads)
        drv = cls(cfg, cols, device, P, forcing, grid=grid, **kw)
        drv.t, drv.step_index = t0, step
        drv.perm, drv.cols_index = perm, idx
        return drv

    def to_grid_order(self, a: np.ndarray) -> np.ndarray:
        """(..., n) columns of the whole set in engine order -> land-point order."""
        perm = getattr(self, "perm", None)
        if perm is None:
            return a
        out = np.empty_like(a)
        out[..., perm] = a
        return out

    # ---- restart -----------------------------------------------------------------
    def save_restart(self, path: str):
        self.ranges.join()
        if path.endswith(".nc"):
            ncio.write_state(path, self.grid, self.to_grid_order(self.cs.state.cpu().numpy()),
                             self.to_grid_order(self.cs.isnow.cpu().numpy()), self.t,
                             self.step_index)
            return
        np.savez(path, time=np.array(self.t.isoformat()), step=np.int64(self.step_index),
                 state=self.cs.state.cpu().numpy(), isnow=self.cs.isnow.cpu().numpy(),
                 static_f=self.cs.static_f.cpu().numpy(), static_i=self.cs.static_i.cpu().numpy(),
                 status=self.cs.status.cpu().numpy(), zsoil=np.asarray(self.zsoil, np.float32),
                 layout=np.array(",".join(n for n, _ in L.STATE_FIELDS)))

    def load_restart(self, path: str):
        self.ranges.join()  # no range may still be stepping the state being replaced
        # the resident LDASIN blocks and the read-ahead belong to the old time:
        # a block kept across a jump could sit in a slot the next upload reuses
        self._blocks.clear()
        if self._prefetch is not None:
            self._prefetch[1].exception()  # a running read-ahead finishes with its buffer
        self._prefetch = None
        if path.endswith(".nc"):
            st, isn, self.t, self.step_index = ncio.read_state(path, self.grid,
                                                               self.cs.state.cpu().numpy().dtype)
            idx = getattr(self, "cols_index", slice(None))
            self.cs.state.copy_(torch.as_tensor(np.ascontiguousarray(st[:, idx]),
                                                device=self.dev))
            self.cs.isnow.copy_(torch.as_tensor(np.ascontiguousarray(isn[idx]), device=self.dev))
            return
        with np.load(path, allow_pickle=False) as z:
            assert str(z["layout"]) == ",".join(n for n, _ in L.STATE_FIELDS), "state layout"
            for name in ("state", "isnow", "static_f", "static_i", "status"):
                getattr(self.cs, name).copy_(torch.as_tensor(z[name], device=self.dev))
            self.t = datetime.datetime.fromisoformat(str(z["time"]))
            self.step_index = int(z["step"])
            self.zsoil = [float(v) for v in z["zsoil"]]

    # ---- time loop -----------------------------------------------------------------
    # the interpreter's thread switch interval while the loop runs: the file
    # reader and writer threads hand the GIL back within this instead of 5 ms
    SWITCH_INTERVAL_S = 0.0005

    def run(self, nsteps: int | None = None):
        import sys
        old = sys.getswitchinterval()
        sys.setswitchinterval(min(old, self.SWITCH_INTERVAL_S))
        try:
            return self._run(nsteps)
        finally:
            sys.setswitchinterval(old)

    def _run(self, nsteps: int | None = None):
        cfg = self.cfg
        total = cfg.step_count() if nsteps is None else nsteps
        rank = dist.get_rank() if dist.is_initialized() else 0
        out_every, res_every = cfg.output_interval, cfg.restart_interval
        for _ in range(total):
            if self.t >= cfg.enddatetime:
                break
            t_iter = time.perf_counter()
            t0 = self.t
            t1 = t0 + cfg.timestep
            out = _is_boundary(t1, cfg.begdatetime, out_every) and self.write
            # the ranges wait for the caller's current stream (state set-up,
            # restart copies, the gather fence assemble() left there) and, for
            # host forcing, for the upload of this step's buffer
            cur = torch.cuda.current_stream(self.dev)
            pre, after, upload, slot = None, (cur, self.upload.stream), self.upload, None
            tp = time.perf_counter()
            # the input file's variable names (header only, once per input time)
            info = self.forcing.variables(t0) if hasattr(self.forcing, "variables") else None
            self.phase_s["read"] += time.perf_counter() - tp
            tp = time.perf_counter()
            if self.raw_upload is not None and not ({"CO2AIR", "O2AIR"} & info):
                # the LDASIN block straight into a pinned buffer and up; each
                # range forms its 12 fields on its own stream before its launch
                step_k, t_k = self.step_index, t0
                geo = solar = None
                if self.geo is not None:
                    # the file's variables go up once per input interval and
                    # stay resident; COSZ is formed on the device every step.
                    # The ranges wait only for their own block's event, so the
                    # next file's upload (enqueued as soon as its bytes are
                    # read) runs beside the steps instead of before one.
                    ti = self.forcing.input_time(t0)
                    if ti not in self._blocks:
                        self._blocks[ti] = self._put_block(t_k, "COSZ" in info)
                    for k in [k for k in self._blocks if k < ti]:
                        del self._blocks[k]
                    raw, ready, upload, slot = self._blocks[ti]
                    if "COSZ" not in info:
                        geo = self.geo
                        solar = timeman.solar_terms(timeman.julian(t0), timeman.yearlen(t0.year))
                    after = (cur, ready)
                else:
                    raw = self.raw_upload.put(fill=lambda h: self.forcing.raw(step_k, t_k, out=h))
                    upload = self.raw_upload
                    after = (cur, upload.stream)
                f = self.raw_fbuf[self.step_index % 2]
                pre = lambda st, rng: self.engine.forcing_from_ldasin(  # noqa: E731
                    raw, f, stream=st, cols=rng, geo=geo, solar=solar)
            elif self.dev_forcing is not None:
                clim, fbuf = self.dev_forcing
                f = fbuf[self.step_index % 2]
                jul, yl, k = timeman.julian(t0), timeman.yearlen(t0.year), self.step_index
                pre = lambda st, rng: self.engine.forcing_synth(  # noqa: E731
                    clim, jul, yl, self.forcing.seed, k, f, self.forcing.first_col, stream=st,
                    cols=rng)
                after, upload = cur, None
            elif info is not None:  # LDASIN files, the 12-field form: built into the pinned buffer
                step_k, t_k = self.step_index, t0
                f = self.upload.put(fill=lambda h: self.forcing(step_k, t_k, out=h))
            else:
                f = self.upload.put(self.forcing(self.step_index, t0))
            self.phase_s["forcing"] += time.perf_counter() - tp
            tp = time.perf_counter()
            diag = self.diag
            if out and self.gather is not None:
                b = self.n_out % len(self.gather.bufs)
                self.gather.release(b, self.ranges.streams)
                diag = self.gather.local(b)
            if out and self._diag_free is not None:
                # the output stream's last read of the diagnostics buffer
                after = (after if isinstance(after, tuple) else (after,)) + (self._diag_free,)
            self.ranges.step(f, self.zsoil, self.dt, timeman.julian(t0), timeman.yearlen(t0.year),
                             diag if out else None, L.DIAG_OUT_LEVEL if out else L.DIAG_NONE,
                             after=after, pre=pre)
            if upload is not None:
                upload.consumed_by(self.ranges.producers, slot)
            if self.geo is not None and self.ingest is not None:
                self._put_next_block(t0)
            self.phase_s["launch"] += time.perf_counter() - tp
            tp = time.perf_counter()
            self.t, self.step_index = t1, self.step_index + 1
            if out:
                if self.gather is not None:
                    self.gather.start(b, producers=self.ranges.producers)
                    d = self.gather.assemble(b)
                    self.n_out += 1
                    ost = torch.cuda.current_stream(self.dev)
                else:
                    # single rank: the output's grids and copy run on their own
                    # stream after this step, beside the next steps
                    if self.out_stream is None:
                        self.out_stream = torch.cuda.Stream(self.dev)
                    ost = self.out_stream
                    self.ranges.join(ost)
                    d = self.diag
                if rank == 0:
                    os.makedirs(cfg.outdir, exist_ok=True)
                    path = (ncio.ldasout_path(cfg.outdir, t1) if self.grid is not None else
                            os.path.join(cfg.outdir, f"{_stamp(t1)}.LDASOUT.npz"))
                    freed = self._write_output(d, path, t1, ost)
                    if self.gather is None:
                        self._diag_free = freed
                    self.written.append(path)
            self.phase_s["output"] += time.perf_counter() - tp
            if _is_boundary(t1, cfg.begdatetime, res_every) and self.write:
                os.makedirs(cfg.resdir, exist_ok=True)
                name = (f"RESTART.{_stamp(t1)}_DOMAIN1.nc" if self.grid is not None and
                        not dist.is_initialized() else f"RESTART.{_stamp(t1)}.r{rank}.npz")
                self.save_restart(os.path.join(cfg.resdir, name))
            self.phase_s["loop"] += time.perf_counter() - t_iter
        self.ranges.join()
        torch.cuda.synchronize(self.dev)
        self.flush_output()
        return self

    def _put_block(self, t: datetime.datetime, file_cosz: bool):
        """Upload the LDASIN block of t's input file once; returns the device
        block and the ForcingUpload whose stream and slot guard it.  With
        `ingest` (and no COSZ in the file) the file's bytes go up as stored and
        the engine forms the block's rows (nmp_ldasin_ingest on the upload's
        stream); otherwise the host builds the block (ncio block)."""
        if self.ingest is None or file_cosz or not self.forcing.ingestible(t):
            up = self.raw_upload
            blk = up.put(fill=lambda h: self.forcing.block(t, out=h))
            ev = torch.cuda.Event()
            ev.record(up.stream)
            return blk, ev, up, up.last_slot
        up, ti = self.ingest, self.forcing.input_time(t)
        ready = False
        if self._prefetch is not None and self._prefetch[0] == ti:
            # the file's bytes were read while the previous file's steps ran
            ready = self._prefetch[1].exception() is None
        self._prefetch = None
        g = up.put(fill=lambda h: self.forcing.grid_raw(t, out=h), prefilled=ready)
        blk = self.ingest_blk[up.last_slot]
        self.engine.ldasin_ingest(g, self.point, blk, stream=up.stream)
        # read the next input file's bytes ahead (a missing or non-fp32 file
        # fails only the prefetch; its step then takes the plain path)
        nxt = ti + self.forcing.every
        if self._prefetch_pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._prefetch_pool = ThreadPoolExecutor(1)
        self._prefetch = (nxt, up.prefetch(lambda h: self.forcing.grid_raw(nxt, out=h),
                                           self._prefetch_pool))
        ev = torch.cuda.Event()
        ev.record(up.stream)
        return blk, ev, up, up.last_slot

    def _put_next_block(self, t: datetime.datetime):
        """Once the next input file's bytes have been read ahead, upload and
        ingest them (on the upload stream, beside the steps of this
        interval) -- when that file takes the ingest path.  Only the interval
        right after t's: the one after that would take the slot this
        interval's remaining steps still read (two slots)."""
        pf = self._prefetch
        if pf is None or pf[0] in self._blocks or not pf[1].done() or \
                pf[0] != self.forcing.input_time(t) + self.forcing.every:
            return
        nxt = pf[0]
        if pf[1].exception() is not None:
            return  # the boundary step reads it itself (and raises if it must)
        info = self.forcing.variables(nxt)
        if {"CO2AIR", "O2AIR", "COSZ"} & info or not self.forcing.ingestible(nxt):
            return
        self._blocks[nxt] = self._put_block(nxt, False)

    # ---- output -----------------------------------------------------------------
    def _write_output(self, d: torch.Tensor, path: str, t1: datetime.datetime, stream=None):
        """One output step's (16, n) fluxes, written on a background thread:
        on `stream` (after the step that produced them) the engine lays them
        on the file's grids in its byte order (nmp_ldasout_grid)
        and they are copied into the next of OUT_BUFFERS pinned host buffers;
        a writer thread (OUT_WRITERS of them) waits for the copy and writes
        the header and the bytes (ncio.write_ldasout_grids) while the loop
        goes on stepping.  A buffer is reused once its previous file is
        written.  The device work goes on `stream` (default: the current
        one); returns the event after which `d` has been read."""
        stream = stream or torch.cuda.current_stream(self.dev)
        src = d
        if self.grid is not None:
            if self._out_point is None:
                perm = getattr(self, "perm", None)
                idx = np.asarray(self.grid.index)
                self._out_point = torch.as_tensor(
                    (idx if perm is None else idx[perm]).astype(np.int32), device=self.dev)
                npts = self.grid.shape[0] * self.grid.shape[1]
                self._out_dev = torch.empty((L.NDIAG_OUT, npts), device=self.dev,
                                            dtype=torch.int32 if d.dtype == torch.float32
                                            else torch.int64)
            self.engine.ldasout_grid(d, self._out_point, self._out_dev, float(ncio.FILL),
                                     stream=stream)
            src = self._out_dev
        if self._writer is None:
            self._writer_init(tuple(src.shape), src.dtype)
        k = self._n_out_w % len(self._out_host)
        self._n_out_w += 1
        if self._out_fut[k] is not None:
            self._out_fut[k].result()
        h = self._out_host[k]
        if h is None or h.shape != src.shape or h.dtype != src.dtype:
            h = self._out_host[k] = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
        with torch.cuda.stream(stream):
            h.copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)

        def job():
            ev.synchronize()
            a = h.numpy()
            if self.grid is not None:
                ncio.write_ldasout_grids(path, self.grid,
                                         a.view(">f4" if a.itemsize == 4 else ">f8"), t1)
            else:
                np.savez(path, time=np.array(t1.isoformat()),
                         fields=np.array(",".join(L.DIAG_OUT)), diag=a)
        self._out_fut[k] = self._writer.submit(job)
        return ev

    # output files in flight at once (writer threads) and staging buffers: a
    # file's write is a memory copy into the page cache on its own thread
    OUT_WRITERS, OUT_BUFFERS = 2, 3

    def _writer_init(self, shape, dtype=None):
        from concurrent.futures import ThreadPoolExecutor
        self._writer = ThreadPoolExecutor(self.OUT_WRITERS)
        dtype = dtype or self.dtype
        self._out_host = [torch.empty(shape, dtype=dtype, pin_memory=True)
                          for _ in range(self.OUT_BUFFERS)]
        self._out_fut, self._n_out_w = [None] * self.OUT_BUFFERS, 0

    def flush_output(self):
        """Wait until every output file issued so far is written (raises a
        writer's error)."""
        for f in getattr(self, "_out_fut", ()):
            if f is not None:
                f.result()
