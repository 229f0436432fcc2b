"""Python front end of the HIP column engine (drop-in for core/module_noahmp_engine.f90).

`Engine` owns the engine handle (tables on the device + options); column data
are caller-owned torch tensors on the engine's GPU in field-major SoA layout
(see layout.py / include/noahmp_engine.h).  `ColumnState` bundles the arrays
of one column set.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import layout as L
from . import lib as _lib
from .params import Params

MATH_REF, MATH_FAST = 0, 1
# nmp_set_launch_variant: occupancy instantiation of the step kernel
LAUNCH_VARIANTS = {"auto": 0, "small": 1, "full": 2}


def _ptr(t, off: int = 0):
    """Device pointer of t, `off` elements in (a column offset into a field-major array)."""
    return C.c_void_p(t.data_ptr() + off * t.element_size()) if t is not None else C.c_void_p(0)


@dataclass
class ColumnState:
    """Device-resident SoA arrays for ncol columns (leading dimension ncol)."""
    state: torch.Tensor     # (56, n) real
    isnow: torch.Tensor     # (n,) int32
    static_f: torch.Tensor  # (6, n) real
    static_i: torch.Tensor  # (6, n) int32
    status: torch.Tensor    # (n,) int32

    @property
    def ncol(self) -> int:
        return int(self.isnow.shape[0])

    @classmethod
    def from_host(cls, cols, device, dtype=torch.float32) -> "ColumnState":
        """From a cases.ColumnSet (numpy SoA)."""
        dev = torch.device(device)
        return cls(
            state=torch.as_tensor(np.ascontiguousarray(cols.state), device=dev).to(dtype).contiguous(),
            isnow=torch.as_tensor(np.ascontiguousarray(cols.isnow, np.int32), device=dev),
            static_f=torch.as_tensor(np.ascontiguousarray(cols.static_f), device=dev).to(dtype).contiguous(),
            static_i=torch.as_tensor(np.ascontiguousarray(cols.static_i, np.int32), device=dev),
            status=torch.zeros(cols.isnow.shape[0], dtype=torch.int32, device=dev),
        )

    def narrow(self, start: int, length: int) -> "ColumnState":
        """A contiguous copy of a column range (for sharding)."""
        return ColumnState(self.state[:, start:start + length].contiguous(),
                           self.isnow[start:start + length].contiguous(),
                           self.static_f[:, start:start + length].contiguous(),
                           self.static_i[:, start:start + length].contiguous(),
                           self.status[start:start + length].contiguous())


class Engine:
    """One engine per device: noahmp_init + *_readptable + noahmp_set_options."""

    def __init__(self, params: Params | None = None, options: dict | None = None,
                 device: int = 0, precision: int = 4, math: int | str = MATH_REF):
        self._lib = _lib.load()
        self.params = params if params is not None else Params.builtin()
        opts = dict(L.CASE_NML_OPTIONS)
        if options:
            opts.update(options)
        self.options = opts
        self.device = int(device)
        self.precision = int(precision)
        self.dtype = torch.float32 if precision == 4 else torch.float64
        o = _lib.NmpOptions(*[int(opts[k]) for k in _lib.NMP_OPTION_FIELDS])
        h = C.c_void_p()
        _lib.check(self._lib.nmp_init(C.byref(self.params.struct), C.byref(o), self.device,
                                      self.precision, C.byref(h)), "nmp_init")
        self._h = h
        if isinstance(math, str):
            math = MATH_FAST if math == "fast" else MATH_REF
        self.set_math(math)

    def set_cols_per_wave(self, cpw: int):
        """nmp_set_cols_per_wave: 8..64 columns per wave, 0 = 64 (default)."""
        _lib.check(self._lib.nmp_set_cols_per_wave(self._h, int(cpw)), "nmp_set_cols_per_wave")

    def option_set(self, request: int = -1) -> int:
        """nmp_option_set: the compiled option set the kernel runs (0 = the
        run-time-options kernel); request 0 forces set 0, 1 picks the match."""
        rc = self._lib.nmp_option_set(self._h, int(request))
        _lib.check(min(rc, 0), "nmp_option_set")
        return rc

    def launch_variant(self, variant: str | int | None = None) -> str:
        """nmp_set_launch_variant: "small" / "full" force the half- / full-
        occupancy kernel for every launch, "auto" (default) picks by column
        count; None only queries.  Returns the variant in use."""
        v = -1 if variant is None else LAUNCH_VARIANTS.get(variant, variant)
        rc = self._lib.nmp_set_launch_variant(self._h, int(v))
        _lib.check(min(rc, 0), "nmp_set_launch_variant")
        return {i: k for k, i in LAUNCH_VARIANTS.items()}[rc]

    def set_math(self, mode: int):
        _lib.check(self._lib.nmp_set_math(self._h, int(mode)), "nmp_set_math")
        self.math = int(mode)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.nmp_finalize(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------------
    def _check_cols(self, cs: ColumnState, forcing: torch.Tensor):
        n = cs.ncol
        assert cs.state.shape == (L.NSTATE, n) and cs.state.dtype == self.dtype
        assert cs.state.is_contiguous() and cs.static_f.is_contiguous()
        assert cs.static_f.shape == (L.NSTATIC_F, n) and cs.static_f.dtype == self.dtype
        assert cs.static_i.shape == (L.NSTATIC_I, n) and cs.static_i.dtype == torch.int32
        assert cs.isnow.dtype == torch.int32 and cs.status.dtype == torch.int32
        assert forcing.shape[-2:] == (L.NFORCING, n) and forcing.dtype == self.dtype
        assert forcing.is_contiguous()
        for t in (cs.state, cs.isnow, cs.static_f, cs.static_i, cs.status, forcing):
            assert t.device.type == "cuda" and t.device.index == self.device, t.device

    def step(self, cs: ColumnState, forcing: torch.Tensor, zsoil, dt: float, julian: float,
             yearlen: int, diag: torch.Tensor | None = None, diag_level: int = L.DIAG_NONE,
             stream=None, cols: tuple[int, int] | None = None, order: torch.Tensor | None = None,
             cost: torch.Tensor | None = None):
        """One noahmp_sflx step for every column (enqueued on `stream`).

        cols=(lo, hi) steps only columns lo..hi-1, in place (pointer offsets with
        ld = cs.ncol; forcing and diag are indexed by the same columns), so
        column ranges can be stepped on different streams.

        order / cost (re-binning, nmp_step_binned): int32 / uint8 tensors of
        cs.ncol entries; the range's slice of `order` must hold a permutation of
        0..hi-lo-1 (indices relative to lo), `cost` receives each column's
        vege_flux trip count."""
        self._check_cols(cs, forcing)
        n = cs.ncol
        lo, hi = (0, n) if cols is None else (int(cols[0]), int(cols[1]))
        assert 0 <= lo <= hi <= n
        if diag_level != L.DIAG_NONE:
            nd = L.NDIAG_FULL if diag_level == L.DIAG_FULL_LEVEL else L.NDIAG_OUT
            assert diag is not None and diag.shape == (nd, n) and diag.dtype == self.dtype
            # raw pointers offset by `lo` with rows exactly n apart: a strided view
            # would be written in the wrong places
            assert diag.is_contiguous()
            assert diag.device.type == "cuda" and diag.device.index == self.device, diag.device
        zs = (C.c_float * 4)(*[float(z) for z in zsoil])
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if order is not None or cost is not None:
            for t, dt_ in ((order, torch.int32), (cost, torch.uint8)):
                if t is not None:
                    assert t.shape == (n,) and t.dtype == dt_ and t.is_contiguous()
                    assert t.device.type == "cuda" and t.device.index == self.device
            if order is not None and os.environ.get("NMP_CHECK_ORDER") == "1":
                # nmp_step_binned trusts order to be a permutation (noahmp_engine.h);
                # the debug check costs a sort and a host sync per launch
                with torch.cuda.stream(s):
                    srt = torch.sort(order[lo:hi])[0]
                    ok = bool(torch.equal(srt, torch.arange(hi - lo, dtype=torch.int32,
                                                            device=order.device)))
                if not ok:
                    raise ValueError(f"order[{lo}:{hi}] is not a permutation of 0..{hi - lo - 1}")
            _lib.check(self._lib.nmp_step_binned(
                self._h, hi - lo, n, zs, float(dt), float(julian), int(yearlen),
                _ptr(cs.state, lo), _ptr(cs.isnow, lo), _ptr(cs.static_f, lo),
                _ptr(cs.static_i, lo), _ptr(forcing, lo), _ptr(diag, lo), int(diag_level),
                _ptr(cs.status, lo), _ptr(order, lo), _ptr(cost, lo),
                C.c_void_p(s.cuda_stream)), "nmp_step_binned")
            return
        _lib.check(self._lib.nmp_step(self._h, hi - lo, n, zs, float(dt), float(julian),
                                      int(yearlen), _ptr(cs.state, lo), _ptr(cs.isnow, lo),
                                      _ptr(cs.static_f, lo), _ptr(cs.static_i, lo),
                                      _ptr(forcing, lo), _ptr(diag, lo), int(diag_level),
                                      _ptr(cs.status, lo), C.c_void_p(s.cuda_stream)), "nmp_step")

    def rebin(self, cost: torch.Tensor, order: torch.Tensor, tile: int, stream=None,
              cols: tuple[int, int] | None = None):
        """nmp_rebin: order[lo:hi] <- the columns lo..hi-1 sorted by cost within
        tiles of `tile` columns (indices relative to lo)."""
        n = int(cost.shape[0])
        lo, hi = (0, n) if cols is None else (int(cols[0]), int(cols[1]))
        assert cost.dtype == torch.uint8 and order.dtype == torch.int32 and order.shape == (n,)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(self._lib.nmp_rebin(self._h, hi - lo, _ptr(cost, lo), _ptr(order, lo),
                                       int(tile), C.c_void_p(s.cuda_stream)), "nmp_rebin")

    def forcing_synth(self, climate: torch.Tensor, julian: float, yearlen: int, seed: int,
                      step: int, out: torch.Tensor, first_col: int = 0, stream=None,
                      cols: tuple[int, int] | None = None):
        """nmp_forcing_synth: one step of synthetic forcing, generated on the
        device from the (NCLIM, n) climate records into out (NFORCING, n);
        cols=(lo, hi) generates only those columns (first_col + lo is their
        global index, so ranges and ranks draw the same numbers as one launch)."""
        n = int(climate.shape[1])
        lo, hi = (0, n) if cols is None else (int(cols[0]), int(cols[1]))
        assert climate.shape == (L.NCLIM, n) and climate.dtype == self.dtype
        assert out.shape == (L.NFORCING, n) and out.dtype == self.dtype
        assert climate.is_contiguous() and out.is_contiguous()
        for t in (climate, out):
            assert t.device.type == "cuda" and t.device.index == self.device
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(self._lib.nmp_forcing_synth(self._h, hi - lo, n, _ptr(climate, lo),
                                               float(julian), int(yearlen), int(seed) & (2**64 - 1),
                                               int(step), int(first_col) + lo, _ptr(out, lo),
                                               C.c_void_p(s.cuda_stream)), "nmp_forcing_synth")

    def forcing_from_ldasin(self, ldasin: torch.Tensor, out: torch.Tensor, stream=None,
                            cols: tuple[int, int] | None = None, geo: torch.Tensor | None = None,
                            solar: tuple[float, float, float] | None = None):
        """nmp_forcing_from_ldasin: the 12 forcing fields of one step into out
        (NFORCING, n), engine precision, from the (NLDASIN, n) fp32 LDASIN
        block (layout.LDASIN); SFCPRS, CO2AIR and O2AIR formed on the device
        from PSFC.  cols=(lo, hi) converts only those columns.

        geo, solar (nmp_forcing_from_ldasin_geo): COSZ formed on the device from
        geo = (3, n) float64 (sin lat, cos lat, lon; ncio.LdasinForcing.geo)
        and solar = timeman.solar_terms(julian, yearlen) instead of read from
        the block's COSZ row."""
        n = int(ldasin.shape[1])
        lo, hi = (0, n) if cols is None else (int(cols[0]), int(cols[1]))
        assert 0 <= lo <= hi <= n
        assert ldasin.shape == (L.NLDASIN, n) and ldasin.dtype == torch.float32
        assert out.shape == (L.NFORCING, n) and out.dtype == self.dtype
        assert ldasin.is_contiguous() and out.is_contiguous()
        for t in (ldasin, out) + ((geo,) if geo is not None else ()):
            assert t.device.type == "cuda" and t.device.index == self.device
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if geo is None:
            _lib.check(self._lib.nmp_forcing_from_ldasin(self._h, hi - lo, n, _ptr(ldasin, lo),
                                                         _ptr(out, lo), C.c_void_p(s.cuda_stream)),
                       "nmp_forcing_from_ldasin")
            return
        assert geo.shape == (3, n) and geo.dtype == torch.float64 and geo.is_contiguous()
        sd, cd, ha0 = (float(v) for v in solar)
        _lib.check(self._lib.nmp_forcing_from_ldasin_geo(
            self._h, hi - lo, n, _ptr(ldasin, lo), _ptr(geo, lo), sd, cd, ha0, _ptr(out, lo),
            C.c_void_p(s.cuda_stream)), "nmp_forcing_from_ldasin_geo")

    def ldasin_ingest(self, grid_be: torch.Tensor, point: torch.Tensor, out: torch.Tensor,
                      stream=None):
        """nmp_ldasin_ingest: rows T2D..LWDOWN of the (NLDASIN, n) fp32 block
        `out` from an LDASIN file's bytes: grid_be = (8, npts) 4-byte words,
        the file's big-endian fp32 grids in layout.LDASIN order; column c takes
        grid point point[c] (int32, (n,)).  The COSZ row is left as it is."""
        n = int(out.shape[1])
        assert grid_be.dim() == 2 and grid_be.shape[0] == L.NLDASIN - 1
        assert grid_be.element_size() == 4 and grid_be.is_contiguous()
        assert point.shape == (n,) and point.dtype == torch.int32 and point.is_contiguous()
        assert out.shape == (L.NLDASIN, n) and out.dtype == torch.float32 and out.is_contiguous()
        for t in (grid_be, point, out):
            assert t.device.type == "cuda" and t.device.index == self.device
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(self._lib.nmp_ldasin_ingest(self._h, n, n, int(grid_be.shape[1]),
                                               _ptr(grid_be, 0), _ptr(point, 0), _ptr(out, 0),
                                               C.c_void_p(s.cuda_stream)), "nmp_ldasin_ingest")

    def ldasout_grid(self, diag: torch.Tensor, point: torch.Tensor, out: torch.Tensor,
                     fill: float, stream=None):
        """nmp_ldasout_grid: the (nfield, n) diagnostics `diag` (engine
        precision) onto out = (nfield, npts) words of the engine's size, the
        file's big-endian grids, `fill` off the columns' points (point: int32
        (n,))."""
        nf, n = int(diag.shape[0]), int(diag.shape[1])
        assert diag.dtype == self.dtype and diag.is_contiguous()
        assert point.shape == (n,) and point.dtype == torch.int32 and point.is_contiguous()
        assert out.dim() == 2 and out.shape[0] == nf and out.is_contiguous()
        assert out.element_size() == self.precision
        for t in (diag, point, out):
            assert t.device.type == "cuda" and t.device.index == self.device
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(self._lib.nmp_ldasout_grid(self._h, n, n, int(out.shape[1]), nf, _ptr(diag, 0),
                                              _ptr(point, 0), float(fill), _ptr(out, 0),
                                              C.c_void_p(s.cuda_stream)), "nmp_ldasout_grid")

    # ---- the reference's other public routines (nmp_frh2o / nmp_calhum) ------
    def frh2o(self, sltyp, tkelv, smc, sh2o, status=None, stream=None):
        """frh2o (func.f90:4494-4598) elementwise.  Device tensors (engine
        precision, int32 sltyp) -> a new tensor of FREE, enqueued on `stream`;
        numpy arrays -> numpy (nmp_frh2o_host, synchronous).  `status` (int32,
        same kind as the inputs) receives NMP_ST_FLERCH / NMP_ST_STOP bits."""
        n = int(len(tkelv))
        if isinstance(tkelv, np.ndarray):
            rt = np.float32 if self.precision == 4 else np.float64
            a = [np.ascontiguousarray(x, rt) for x in (tkelv, smc, sh2o)]
            si = np.ascontiguousarray(sltyp, np.int32)
            # the library copies n elements of every array: a shorter one would be over-read
            for x in (*a, si):
                assert x.shape == (n,), f"frh2o: every input must have shape ({n},), got {x.shape}"
            out = np.empty(n, rt)
            st = status if status is not None else np.zeros(n, np.int32)
            assert st.dtype == np.int32 and st.flags.c_contiguous and st.shape == (n,)
            _lib.check(self._lib.nmp_frh2o_host(self._h, n, C.c_void_p(si.ctypes.data),
                                                *[C.c_void_p(x.ctypes.data) for x in a],
                                                C.c_void_p(out.ctypes.data),
                                                C.c_void_p(st.ctypes.data)), "nmp_frh2o_host")
            return out
        for t in (tkelv, smc, sh2o):
            assert t.dtype == self.dtype and t.is_contiguous() and t.shape == (n,)
            assert t.device.type == "cuda" and t.device.index == self.device
        assert sltyp.dtype == torch.int32 and sltyp.is_contiguous() and sltyp.shape == (n,)
        assert sltyp.device.type == "cuda" and sltyp.device.index == self.device, sltyp.device
        if status is not None:
            # the kernel ORs int32 bits into n elements of it on the device
            assert status.dtype == torch.int32 and status.is_contiguous() and status.shape == (n,)
            assert status.device.type == "cuda" and status.device.index == self.device
        out = torch.empty(n, dtype=self.dtype, device=tkelv.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(self._lib.nmp_frh2o(self._h, n, _ptr(sltyp), _ptr(tkelv), _ptr(smc), _ptr(sh2o),
                                       _ptr(out), _ptr(status), C.c_void_p(s.cuda_stream)),
                   "nmp_frh2o")
        return out

    def calhum(self, sfctmp, sfcprs, stream=None):
        """calhum (func.f90:3958-3984) elementwise -> (Q2SAT, DQSDT2); device
        tensors (enqueued on `stream`) or numpy arrays (synchronous)."""
        n = int(len(sfctmp))
        if isinstance(sfctmp, np.ndarray):
            rt = np.float32 if self.precision == 4 else np.float64
            t, p = (np.ascontiguousarray(x, rt) for x in (sfctmp, sfcprs))
            assert t.shape == p.shape == (n,), f"calhum: inputs must have shape ({n},)"
            q, d = np.empty(n, rt), np.empty(n, rt)
            _lib.check(self._lib.nmp_calhum_host(self._h, n, C.c_void_p(t.ctypes.data),
                                                 C.c_void_p(p.ctypes.data), C.c_void_p(q.ctypes.data),
                                                 C.c_void_p(d.ctypes.data)), "nmp_calhum_host")
            return q, d
        for x in (sfctmp, sfcprs):
            assert x.dtype == self.dtype and x.is_contiguous() and x.shape == (n,)
            assert x.device.type == "cuda" and x.device.index == self.device
        q = torch.empty(n, dtype=self.dtype, device=sfctmp.device)
        d = torch.empty_like(q)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(self._lib.nmp_calhum(self._h, n, _ptr(sfctmp), _ptr(sfcprs), _ptr(q), _ptr(d),
                                        C.c_void_p(s.cuda_stream)), "nmp_calhum")
        return q, d

    def sflx_columns(self, rec: np.ndarray) -> np.ndarray:
        """noahmp_sflx with the reference calling sequence on host records
        (layout.sflx_args_dtype(); nmp_sflx_columns), updated in place and returned.
        Synchronous: packs, steps on the engine's GPU, unpacks."""
        assert rec.dtype == L.sflx_args_dtype() and rec.flags.c_contiguous and rec.ndim == 1
        _lib.check(self._lib.nmp_sflx_columns(self._h, C.c_void_p(rec.ctypes.data),
                                              int(rec.shape[0])), "nmp_sflx_columns")
        return rec

    def run(self, cs: ColumnState, forcings: torch.Tensor, zsoil, dt: float, julian0: float,
            yearlen: int, nsteps: int, diag: torch.Tensor | None = None,
            diag_level: int = L.DIAG_NONE, stream=None, out_every: int | None = None):
        """nsteps steps in one launch, cycling through forcings[(period, 12, n)].

        Diagnostics: with `out_every` None, `diag` (nd, n) receives the last step
        (nmp_run); otherwise every out_every-th step writes the next slot of the
        ring `diag` (slots, nd, n), wrapping (nmp_run_out)."""
        n = cs.ncol
        assert forcings.dim() == 3
        self._check_cols(cs, forcings[0])
        zs = (C.c_float * 4)(*[float(z) for z in zsoil])
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if diag_level != L.DIAG_NONE:
            nd = L.NDIAG_FULL if diag_level == L.DIAG_FULL_LEVEL else L.NDIAG_OUT
            assert diag is not None and diag.dtype == self.dtype and diag.is_contiguous()
            assert diag.shape[-2:] == (nd, n) and diag.dim() == (2 if out_every is None else 3)
            assert diag.device.type == "cuda" and diag.device.index == self.device
        if out_every is None:
            _lib.check(self._lib.nmp_run(self._h, n, n, zs, float(dt), float(julian0), int(yearlen),
                                         int(nsteps), _ptr(cs.state), _ptr(cs.isnow),
                                         _ptr(cs.static_f), _ptr(cs.static_i), _ptr(forcings),
                                         L.NFORCING * n, forcings.shape[0], _ptr(diag),
                                         int(diag_level), _ptr(cs.status),
                                         C.c_void_p(s.cuda_stream)), "nmp_run")
            return
        slots = diag.shape[0] if diag is not None else 1
        dstride = diag[0].numel() if diag is not None else 0
        _lib.check(self._lib.nmp_run_out(self._h, n, n, zs, float(dt), float(julian0),
                                         int(yearlen), int(nsteps), _ptr(cs.state),
                                         _ptr(cs.isnow), _ptr(cs.static_f), _ptr(cs.static_i),
                                         _ptr(forcings), L.NFORCING * n, forcings.shape[0],
                                         _ptr(diag), int(diag_level), int(out_every), int(slots),
                                         int(dstride), _ptr(cs.status),
                                         C.c_void_p(s.cuda_stream)), "nmp_run_out")


class StreamShards:
    """Steps one ColumnState as `nshards` column ranges, each on its own HIP stream.

    Columns are independent and a range's step t+1 depends only on its own step
    t, so the ranges' launches need no synchronisation with each other.  While
    one range's launch drains its last waves, the other range's waves fill the
    idle SIMDs, which hides the per-launch tail (DESIGN.md "Launch structure").
    `join()` makes a stream wait for every range, and is needed before the
    caller reads state or diagnostics."""

    def __init__(self, engine: Engine, cs: ColumnState, nshards: int = 2, device=None,
                 rebin_tile: int = 0, rebin_every: int = 1, launch_cols: int = 0,
                 first_frac: float | None = None, stagger: bool = False):
        """rebin_tile > 0 turns on column re-binning (nmp_step_binned /
        nmp_rebin): every `rebin_every` steps each range re-sorts its columns
        within tiles of rebin_tile columns by the trip counts the previous step
        recorded, and the next launches step them in that order.
        launch_cols > 0 (launch-size study): each range is stepped as
        sequential launches of at most launch_cols columns on its stream.
        first_frac (two ranges only): the first range's share of the columns
        (default: equal ranges).  stagger: the first step of range i > 0 starts
        after range i - 1's first launch, so the ranges run out of phase (their
        launches' ramp and drain fall on the other range's full waves)."""
        n = cs.ncol
        nshards = max(1, min(int(nshards), max(n, 1)))
        self.engine, self.cs = engine, cs
        dev = torch.device("cuda", engine.device) if device is None else torch.device(device)
        self.streams = [torch.cuda.Stream(dev) for _ in range(nshards)]
        self.ranges = [(n * i // nshards, n * (i + 1) // nshards) for i in range(nshards)]
        if first_frac is not None and nshards == 2:
            cut = min(max(int(round(n * first_frac)) // 256 * 256, 0), n)
            self.ranges = [(0, cut), (cut, n)]
        self.rebin_tile, self.rebin_every, self.nstep = int(rebin_tile), max(1, int(rebin_every)), 0
        self.launch_cols = int(launch_cols)
        self.stagger, self._stag_ev = bool(stagger), None
        assert not (self.launch_cols and self.rebin_tile), "launch_cols: plain launches only"
        self.order = self.cost = None
        if self.rebin_tile:
            # identity order to start with, relative to each range's first column
            self.order = torch.cat([torch.arange(hi - lo, dtype=torch.int32)
                                    for lo, hi in self.ranges]).to(dev) if n else \
                torch.zeros(0, dtype=torch.int32, device=dev)
            self.cost = torch.zeros(n, dtype=torch.uint8, device=dev)

    def step(self, forcing: torch.Tensor, zsoil, dt: float, julian: float, yearlen: int,
             diag: torch.Tensor | None = None, diag_level: int = L.DIAG_NONE, events=None,
             after="current", pre=None):
        """One step of every range.  `after`: the stream, or a tuple of streams
        and events, whose pending work (the forcing upload, a previous reader
        of `diag`) each range waits for first -- by default the caller's current stream,
        where torch enqueues uploads; tensors are kept alive until the ranges
        are done with them.  Pass None only when the inputs are known to be
        complete (e.g. after a synchronize).
        events: per-range (start, end) pairs.  pre(stream, (lo, hi)): work
        enqueued on each range's stream before its step (e.g. generating that
        range's forcing on the device, Engine.forcing_synth)."""
        if isinstance(after, str) and after == "current":
            after = torch.cuda.current_stream(self.streams[0].device)
        if after is not None and not isinstance(after, (tuple, list)):
            after = (after,)
        for i, (st, rng) in enumerate(zip(self.streams, self.ranges)):
            if after is not None:
                for a in after:
                    if isinstance(a, torch.cuda.Event):
                        st.wait_event(a)
                    else:
                        st.wait_stream(a)
                forcing.record_stream(st)
                if diag is not None:
                    diag.record_stream(st)
            if self.stagger and self.nstep == 0 and i > 0:
                st.wait_event(self._stag_ev)
            if pre is not None:
                pre(st, rng)
            if events is not None:
                events[i][0].record(st)
            if self.rebin_tile and self.nstep > 0 and self.nstep % self.rebin_every == 0:
                self.engine.rebin(self.cost, self.order, self.rebin_tile, stream=st, cols=rng)
            if self.launch_cols:
                for lo in range(rng[0], rng[1], self.launch_cols):
                    self.engine.step(self.cs, forcing, zsoil, dt, julian, yearlen, diag,
                                     diag_level, stream=st,
                                     cols=(lo, min(lo + self.launch_cols, rng[1])))
            else:
                self.engine.step(self.cs, forcing, zsoil, dt, julian, yearlen, diag, diag_level,
                                 stream=st, cols=None if len(self.streams) == 1 else rng,
                                 order=self.order, cost=self.cost)
            if events is not None:
                events[i][1].record(st)
            if self.stagger and self.nstep == 0:
                self._stag_ev = torch.cuda.Event()
                self._stag_ev.record(st)
        self.nstep += 1

    @property
    def producers(self):
        """Every stream that writes the ranges' state and diagnostics."""
        return list(self.streams)

    def join(self, stream: torch.cuda.Stream | None = None):
        """Make `stream` (default: the current stream) wait for every range."""
        s = stream if stream is not None else torch.cuda.current_stream(self.streams[0].device)
        for st in self.producers:
            s.wait_stream(st)
