"""netCDF-3 files of the offline run: static grid, initial/restart state,
LDASIN forcing and LDASOUT output.

The reference names these files in its namelist (run/case.nml:2-11:
static_parameter_file, initialization_file, restart_file, input_directory,
output_directory) but ships no reader or writer for them (run/main.py stops
after the namelist).  This module supplies them in the
HRLDAS conventions Noah-MP offline runs use, as netCDF-3 classic files through
scipy.io.netcdf_file (no netCDF-4/HDF5 library exists in this image):

* static file (geo_em-style), dims (south_north, west_east[, month]):
  XLAT_M, XLONG_M (deg), LANDMASK, LU_INDEX (vegetation type), SCT_DOM (soil
  type), SLOPECAT, SOILCOLOR, SOILTEMP (deep soil T -> TBOT), GREENFRAC
  (12 monthly fractions -> SHDFAC by the date), SHDMAX (default: the
  GREENFRAC maximum), ZLVL, FOLN,
  ISLAKE/ISICE from the table's ISWATER/ISICE types;
* LDASIN, one file per input time, ``<YYYYMMDDHH>.LDASIN_DOMAIN1``:
  T2D, Q2D, U2D, V2D, PSFC, RAINRATE, SWDOWN, LWDOWN on (Time, south_north,
  west_east).  Optional extras COSZ, CO2AIR, O2AIR override the derived values
  (COSZ from the grid's lat/lon at the step's time, CO2AIR = 395e-6 PSFC,
  O2AIR = 0.209 PSFC);
* state file (initialization_file / restart_file): the engine's SoA state,
  one variable per state field (layer fields get a layer dimension), ISNOW,
  plus the model time -- the state SoA *is* the restart;
* LDASOUT, one file per output time, ``<YYYYMMDDHH>.LDASOUT_DOMAIN1``: the 16
  output fluxes on the grid, _FillValue off the land mask.

Columns are the grid's land points (LANDMASK == 1) in row-major order.
"""
from __future__ import annotations

import datetime
import os

import numpy as np
from scipy.io import netcdf_file

from . import cases, layout as L, timeman

FILL = np.float32(-9999.0)
LDASIN_MAP = {"SFCTMP": "T2D", "Q2": "Q2D", "UU": "U2D", "VV": "V2D", "SFCPRS": "PSFC",
              "PSFC": "PSFC", "PRCP": "RAINRATE", "SOLDN": "SWDOWN", "LWDN": "LWDOWN"}
LDASIN_UNITS = {"T2D": "K", "Q2D": "kg kg-1", "U2D": "m s-1", "V2D": "m s-1", "PSFC": "Pa",
                "RAINRATE": "kg m-2 s-1", "SWDOWN": "W m-2", "LWDOWN": "W m-2",
                "COSZ": "1", "CO2AIR": "Pa", "O2AIR": "Pa"}
_LAYER_DIMS = {7: "snso_layers", 4: "soil_layers", 3: "snow_layers"}


def stamp(t: datetime.datetime) -> str:
    """HRLDAS file-time stamp YYYYMMDDHH; minutes are appended for off-hour
    times (input or output intervals below an hour)."""
    return t.strftime("%Y%m%d%H" if t.minute == 0 and t.second == 0 else "%Y%m%d%H%M")


def ldasin_path(indir: str, t: datetime.datetime) -> str:
    return os.path.join(indir, f"{stamp(t)}.LDASIN_DOMAIN1")


def ldasout_path(outdir: str, t: datetime.datetime) -> str:
    return os.path.join(outdir, f"{stamp(t)}.LDASOUT_DOMAIN1")


def _read(path: str):
    if not os.path.isfile(path):
        raise FileNotFoundError(path)
    return netcdf_file(path, "r", mmap=False)


# ---- grid -------------------------------------------------------------------------
class Grid:
    """Land points of a (south_north, west_east) grid, row-major."""

    def __init__(self, lat_deg: np.ndarray, lon_deg: np.ndarray, mask: np.ndarray):
        self.shape = tuple(mask.shape)
        self.lat_deg = np.asarray(lat_deg, np.float64)
        self.lon_deg = np.asarray(lon_deg, np.float64)
        self.mask = np.asarray(mask, bool)
        self.index = np.flatnonzero(self.mask.reshape(-1))

    @property
    def n(self) -> int:
        return int(self.index.size)

    def columns(self, field2d: np.ndarray) -> np.ndarray:
        return np.asarray(field2d).reshape(-1)[self.index]

    def scatter(self, cols: np.ndarray, fill=FILL) -> np.ndarray:
        out = np.full(self.shape[0] * self.shape[1], fill, np.asarray(cols).dtype)
        out[self.index] = cols
        return out.reshape(self.shape)

    @property
    def lat_rad(self) -> np.ndarray:
        return np.radians(self.columns(self.lat_deg))

    @property
    def lon_rad(self) -> np.ndarray:
        return np.radians(self.columns(self.lon_deg))


# ---- static file ----------------------------------------------------------------
def write_static(path: str, cols: cases.ColumnSet, grid: Grid, greenfrac=None):
    """A geo_em-style static file for `cols` laid on `grid` (tests / examples)."""
    ny, nx = grid.shape
    f = netcdf_file(path, "w")
    try:
        f.createDimension("south_north", ny)
        f.createDimension("west_east", nx)
        f.createDimension("month", 12)
        dims = ("south_north", "west_east")

        def put(name, data, kind="f4", units=None):
            v = f.createVariable(name, kind, dims)
            v[:] = data
            if units:
                v.units = units

        # f8 degrees: radians -> degrees -> radians returns the columns' f32 LAT exactly
        put("XLAT_M", grid.lat_deg, "f8", units="degrees_north")
        put("XLONG_M", grid.lon_deg, "f8", units="degrees_east")
        put("LANDMASK", grid.mask.astype(np.int32), "i4")
        sf, si = cols.static_f, cols.static_i
        for name, row in (("LU_INDEX", "VEGTYP"), ("SCT_DOM", "SOILTYP"), ("SLOPECAT", "SLOPETYP"),
                          ("SOILCOLOR", "SOILCOLOR")):
            put(name, grid.scatter(si[L.STATIC_I.index(row)].astype(np.int32), 0), "i4")
        put("SOILTEMP", grid.scatter(sf[L.STATIC_F.index("TBOT")]), units="K")
        put("ZLVL", grid.scatter(sf[L.STATIC_F.index("ZLVL")]), units="m")
        put("FOLN", grid.scatter(sf[L.STATIC_F.index("FOLN")]))
        if greenfrac is None:  # constant in time: the columns' SHDFAC every month
            greenfrac = np.repeat(sf[L.STATIC_F.index("SHDFAC")][None, :], 12, 0)
        put("SHDMAX", grid.scatter(sf[L.STATIC_F.index("SHDMAX")]))
        v = f.createVariable("GREENFRAC", "f4", ("month",) + dims)
        v[:] = np.stack([grid.scatter(np.asarray(g, np.float32)) for g in greenfrac])
    finally:
        f.close()


def read_static(path: str, params: dict, when: datetime.datetime):
    """(Grid, static_f (6, n) f32, static_i (6, n) i32) of a static file.
    SHDFAC is GREENFRAC interpolated to `when` (mid-month weights), SHDMAX its
    annual maximum; IST = 2 on the table's water type, ICE = 1 on its ice type."""
    f = _read(path)
    try:
        v = f.variables
        lat, lon = np.array(v["XLAT_M"][:]), np.array(v["XLONG_M"][:])
        mask = np.array(v["LANDMASK"][:]) == 1 if "LANDMASK" in v else np.ones(lat.shape, bool)
        grid = Grid(lat, lon, mask)
        n = grid.n
        col = lambda name, default: (grid.columns(np.array(v[name][:])) if name in v  # noqa: E731
                                     else np.full(n, default))
        lut = col("LU_INDEX", 7).astype(np.int32)
        slt = col("SCT_DOM", 6).astype(np.int32)
        gf = np.array(v["GREENFRAC"][:]) if "GREENFRAC" in v else None
        sf = np.zeros((L.NSTATIC_F, n), np.float32)
        si = np.zeros((L.NSTATIC_I, n), np.int32)
        sf[L.STATIC_F.index("LAT")] = np.radians(grid.columns(lat))
        sf[L.STATIC_F.index("ZLVL")] = col("ZLVL", 10.0)
        sf[L.STATIC_F.index("TBOT")] = col("SOILTEMP", 285.0)
        sf[L.STATIC_F.index("FOLN")] = col("FOLN", 1.0)
        if gf is not None:
            g = np.stack([grid.columns(gf[m]) for m in range(12)])
            sf[L.STATIC_F.index("SHDFAC")] = _month_weighted(g, when)
            sf[L.STATIC_F.index("SHDMAX")] = col("SHDMAX", 0.0) if "SHDMAX" in v else g.max(0)
        else:
            sf[L.STATIC_F.index("SHDFAC")] = 0.7
            sf[L.STATIC_F.index("SHDMAX")] = 0.8
        si[L.STATIC_I.index("VEGTYP")] = lut
        si[L.STATIC_I.index("SOILTYP")] = slt
        si[L.STATIC_I.index("SLOPETYP")] = col("SLOPECAT", 1)
        si[L.STATIC_I.index("SOILCOLOR")] = col("SOILCOLOR", 4)
        si[L.STATIC_I.index("IST")] = np.where(lut == params["iswater"], 2, 1)
        si[L.STATIC_I.index("ICE")] = np.where(lut == params["isice"], 1, 0)
        return grid, sf, si
    finally:
        f.close()


def _month_weighted(g12: np.ndarray, when: datetime.datetime) -> np.ndarray:
    """Linear interpolation between mid-month values (a monthly climatology at `when`)."""
    ylen = timeman.yearlen(when.year)
    t = 12.0 * timeman.julian(when) / ylen - 0.5
    m0 = int(np.floor(t)) % 12
    w = t - np.floor(t)
    return ((1.0 - w) * g12[m0] + w * g12[(m0 + 1) % 12]).astype(np.float32)


# ---- state (initialization / restart) ----------------------------------------------
def write_state(path: str, grid: Grid, state: np.ndarray, isnow: np.ndarray,
                t: datetime.datetime, step: int = 0):
    """SoA state (56, n) + ISNOW on the grid; layer fields get a layer dimension."""
    ny, nx = grid.shape
    f = netcdf_file(path, "w")
    try:
        f.createDimension("south_north", ny)
        f.createDimension("west_east", nx)
        for w, d in _LAYER_DIMS.items():
            f.createDimension(d, w)
        f.model_time = t.isoformat()
        f.model_step = np.int32(step)
        f.state_layout = ",".join(n for n, _ in L.STATE_FIELDS)
        dims = ("south_north", "west_east")
        kind = "f8" if state.dtype == np.float64 else "f4"
        for name, w in L.STATE_FIELDS:
            o = L.STATE_OFF[name][0]
            if w == 1:
                v = f.createVariable(name, kind, dims)
                v[:] = grid.scatter(state[o].astype(kind), np.asarray(FILL, kind))
            else:
                v = f.createVariable(name, kind, (_LAYER_DIMS[w],) + dims)
                v[:] = np.stack([grid.scatter(state[o + k].astype(kind), np.asarray(FILL, kind))
                                 for k in range(w)])
        v = f.createVariable("ISNOW", "i4", dims)
        v[:] = grid.scatter(isnow.astype(np.int32), 0)
    finally:
        f.close()


def read_state(path: str, grid: Grid, dtype=np.float32):
    """(state (56, n), isnow (n,), time, step) from a state file on `grid`."""
    f = _read(path)
    try:
        layout = f.state_layout.decode() if isinstance(f.state_layout, bytes) else f.state_layout
        assert layout == ",".join(n for n, _ in L.STATE_FIELDS), "state layout"
        st = np.zeros((L.NSTATE, grid.n), dtype)
        for name, w in L.STATE_FIELDS:
            o = L.STATE_OFF[name][0]
            a = np.array(f.variables[name][:])
            if w == 1:
                st[o] = grid.columns(a)
            else:
                for k in range(w):
                    st[o + k] = grid.columns(a[k])
        isnow = grid.columns(np.array(f.variables["ISNOW"][:])).astype(np.int32)
        mt = f.model_time.decode() if isinstance(f.model_time, bytes) else f.model_time
        return st, isnow, datetime.datetime.fromisoformat(mt), int(f.model_step)
    finally:
        f.close()


# ---- LDASIN ---------------------------------------------------------------------
def write_ldasin(path: str, grid: Grid, forcing: np.ndarray, t: datetime.datetime,
                 extras=True):
    """One LDASIN file from a (12, n) forcing slice; `extras` (True, or a
    tuple of some of "COSZ", "CO2AIR", "O2AIR") also stores those fields, so
    that with all three the file reproduces the slice exactly."""
    ny, nx = grid.shape
    f = netcdf_file(path, "w")
    try:
        f.createDimension("Time", None)
        f.createDimension("south_north", ny)
        f.createDimension("west_east", nx)
        f.valid_time = t.isoformat()
        dims = ("Time", "south_north", "west_east")
        names = dict(LDASIN_MAP)
        names.pop("SFCPRS")  # SFCPRS and PSFC share the PSFC variable
        for x in (("COSZ", "CO2AIR", "O2AIR") if extras is True else (extras or ())):
            names[x] = x
        for fld, var in names.items():
            v = f.createVariable(var, "f4", dims)
            v[0] = grid.scatter(forcing[L.FORCING.index(fld)].astype(np.float32))
            v.units = LDASIN_UNITS[var]
    finally:
        f.close()


def read_ldasin(path: str) -> dict:
    f = _read(path)
    try:
        return {k: np.array(v[0] if v.dimensions[0] == "Time" else v[:])
                for k, v in f.variables.items()}
    finally:
        f.close()


class LdasinForcing:
    """Forcing provider for driver.OfflineDriver from LDASIN files: the file of
    the latest input time <= the step's start time (input_frequency, counted
    from the run's start), held constant over the input interval.

    Two forms: `__call__` gives the 12 noahmp_sflx forcing fields built on the
    host; `raw` gives the LDASIN block as the files carry it (the 8 variables
    plus the step's COSZ, fp32, layout.LDASIN order), from which the engine
    forms the other fields on the device (nmp_forcing_from_ldasin) -- a third
    fewer bytes to build and upload per step, the same values.

    Both are filled by `threads` host threads over column chunks (numpy
    releases the GIL in its elementwise loops); every element is computed by
    the same expression as in one pass, so the values do not depend on it.
    COSZ, a double cosine per column and step, dominated the host's time."""

    def __init__(self, indir: str, grid: Grid, begin: datetime.datetime,
                 every: datetime.timedelta, cols: slice | None = None, threads: int | None = None):
        """cols: the land points this rank steps, in engine order (a slice or an
        index array; default: all of them in grid order).  threads: host
        threads (default NMP_HOST_THREADS, else 8)."""
        self.indir, self.grid, self.begin, self.every = indir, grid, begin, every
        self.cols = cols if cols is not None else slice(0, grid.n)
        self._t, self._fields = None, None
        self.lat, self.lon = self.grid.lat_rad[self.cols], self.grid.lon_rad[self.cols]
        # the latitude factors of COSZ, once (timeman.cosz evaluates the same
        # numpy functions on the same values every step)
        self._sincos_lat = (np.sin(self.lat), np.cos(self.lat))
        # file grid point of each engine column: one gather per variable
        self._gidx = np.asarray(grid.index)[self.cols]
        self.threads = max(1, int(threads if threads is not None else
                                  os.environ.get("NMP_HOST_THREADS", 8)))
        # shared by the read-ahead thread (_load) and the caller (_chunks);
        # its threads start on first use
        from concurrent.futures import ThreadPoolExecutor
        self._pool = ThreadPoolExecutor(self.threads) if self.threads > 1 else None

    def input_time(self, t: datetime.datetime) -> datetime.datetime:
        k = (t - self.begin) // self.every
        return self.begin + k * self.every

    def _load(self, ti: datetime.datetime) -> dict:
        """This rank's columns of every variable of the input time's file, in
        engine order and native byte order: one gather per variable straight
        from the mapped file through the composite index (engine column ->
        grid point), the variables on the provider's threads.  The values are
        read_ldasin's, selected by grid.columns and then `cols`."""
        path = ldasin_path(self.indir, ti)
        if not os.path.isfile(path):
            raise FileNotFoundError(path)
        f = netcdf_file(path, "r", mmap=True)
        out = {}
        try:
            names = list(f.variables)

            def one(k):
                v = f.variables[k]
                s = np.asarray(v[0] if v.dimensions[0] == "Time" else v[:]).reshape(-1)
                out[k] = s[self._gidx].astype(s.dtype.newbyteorder("="))
            self._map(one, names)
        finally:
            f.close()
        return out

    def _map(self, fn, items):
        """fn(item) for every item, on the provider's threads."""
        if self._pool is None or len(items) < 2:
            for x in items:
                fn(x)
            return
        for fut in [self._pool.submit(fn, x) for x in items]:
            fut.result()

    def fields(self, t: datetime.datetime) -> dict:
        """The LDASIN variables of the step starting at t (this rank's columns).
        The next input time's file is read ahead on a background thread while
        the steps of this one run (a missing next file only fails when a
        step needs it)."""
        ti = self.input_time(t)
        if ti != self._t:
            ahead = getattr(self, "_ahead", None)
            if ahead is not None and ahead[0] == ti:
                self._fields = ahead[1].result()
            else:
                self._fields = self._load(ti)
            self._t = ti
            if getattr(self, "_reader", None) is None:
                from concurrent.futures import ThreadPoolExecutor
                self._reader = ThreadPoolExecutor(1)
            nxt = ti + self.every
            self._ahead = (nxt, self._reader.submit(self._load, nxt))
        return self._fields

    def _chunks(self, fill):
        """fill(slice) over column chunks, on the provider's threads."""
        n = self.lat.shape[0]
        k = min(self.threads, max(1, n // 65536))
        sl = [slice(n * i // k, n * (i + 1) // k) for i in range(k)]
        self._map(fill, sl)

    def _cosz(self, fl: dict, t: datetime.datetime, c: slice) -> np.ndarray:
        if "COSZ" in fl:
            return fl["COSZ"][c]
        return timeman.cosz(self.lat[c], self.lon[c], timeman.julian(t), timeman.yearlen(t.year),
                            sincos_lat=(self._sincos_lat[0][c], self._sincos_lat[1][c]))

    def __call__(self, step: int, t: datetime.datetime, out: np.ndarray | None = None):
        fl = self.fields(t)
        f = np.empty((L.NFORCING, self.lat.shape[0]), np.float32) if out is None else out
        F = L.FORCING.index

        def fill(c):
            for fld, var in LDASIN_MAP.items():
                f[F(fld), c] = fl[var][c]
            # every field is an fp32 value (the LDASIN precision), also when
            # `out` is an fp64 engine's buffer
            psfc = fl["PSFC"][c].astype(np.float64)
            f32 = np.float32
            f[F("COSZ"), c] = np.asarray(self._cosz(fl, t, c)).astype(f32)
            f[F("CO2AIR"), c] = fl["CO2AIR"][c] if "CO2AIR" in fl else (395.0e-6 * psfc).astype(f32)
            f[F("O2AIR"), c] = fl["O2AIR"][c] if "O2AIR" in fl else (0.209 * psfc).astype(f32)
        self._chunks(fill)
        return f

    def raw(self, step: int, t: datetime.datetime, out: np.ndarray | None = None):
        """(NLDASIN, n) fp32 LDASIN block of the step starting at t, written
        into `out` when given (e.g. a pinned upload buffer); None when the file
        carries CO2AIR / O2AIR of its own (then only the 12-field form holds
        them)."""
        fl = self.fields(t)
        if "CO2AIR" in fl or "O2AIR" in fl:
            return None
        r = np.empty((L.NLDASIN, self.lat.shape[0]), np.float32) if out is None else out

        def fill(c):
            for i, var in enumerate(L.LDASIN):
                r[i, c] = self._cosz(fl, t, c) if var == "COSZ" else fl[var][c]
        self._chunks(fill)
        return r

    def block(self, t: datetime.datetime, out: np.ndarray | None = None):
        """The LDASIN block of the input interval holding t without the
        per-step COSZ: the 8 file variables (and the file's own COSZ when it
        carries one; else that row is left as it is), for a host that uploads
        them once per input interval and forms COSZ on the device
        (nmp_forcing_from_ldasin_geo with `geo`).  None when the file carries
        CO2AIR / O2AIR of its own."""
        fl = self.fields(t)
        if "CO2AIR" in fl or "O2AIR" in fl:
            return None
        r = np.empty((L.NLDASIN, self.lat.shape[0]), np.float32) if out is None else out
        rows = [(i, v) for i, v in enumerate(L.LDASIN) if v != "COSZ" or "COSZ" in fl]

        def fill(c):
            for i, var in rows:
                r[i, c] = fl[var][c]
        self._chunks(fill)
        return r

    def variables(self, t: datetime.datetime) -> frozenset:
        """The variable names of the input file of t (its header only, cached
        per input time)."""
        ti = self.input_time(t)
        cache = self.__dict__.setdefault("_vars_cache", {})
        if ti in cache:
            self._vars_t, (self._vars, self._ingestible) = ti, cache[ti]
        if getattr(self, "_vars_t", None) != ti:
            path = ldasin_path(self.indir, ti)
            if not os.path.isfile(path):
                raise FileNotFoundError(path)
            f = netcdf_file(path, "r", mmap=True)
            try:
                self._vars = frozenset(f.variables)
                # the device ingest takes the 8 variables as fp32 grids
                npts = self.grid.shape[0] * self.grid.shape[1]
                self._ingestible = all(
                    k in f.variables and f.variables[k].data.dtype == np.dtype(">f4") and
                    f.variables[k].data.size in (npts, npts * f.variables[k].data.shape[0])
                    and f.variables[k].data.shape[-2:] == self.grid.shape
                    for k in L.LDASIN[:-1])
            finally:
                f.close()
            self._vars_t = ti
            cache[ti] = (self._vars, self._ingestible)
            while len(cache) > 4:   # the current and next input times, a few back
                del cache[min(cache)]
        return self._vars

    def ingestible(self, t: datetime.datetime) -> bool:
        """The input file of t holds the 8 LDASIN variables as fp32 grids of
        the run's shape (what grid_raw / nmp_ldasin_ingest take)."""
        self.variables(t)
        return self._ingestible

    def point(self) -> np.ndarray:
        """int32 (n,): the file grid point (row-major index) of each engine
        column -- nmp_ldasin_ingest's `point`."""
        return self._gidx.astype(np.int32)

    def grid_raw(self, t: datetime.datetime, out: np.ndarray | None = None):
        """The input file's 8 LDASIN variables (layout.LDASIN order, COSZ
        excluded) as the file stores them: (8, npts) big-endian fp32 grids,
        copied byte for byte into `out` (any 4-byte dtype, e.g. a pinned
        upload buffer's int32 view), one variable per provider thread.  The
        engine selects this rank's columns, applies its order and the byte
        order on the device (nmp_ldasin_ingest)."""
        path = ldasin_path(self.indir, self.input_time(t))
        if not os.path.isfile(path):
            raise FileNotFoundError(path)
        npts = self.grid.shape[0] * self.grid.shape[1]
        r = np.empty((L.NLDASIN - 1, npts), ">f4") if out is None else out
        assert r.shape == (L.NLDASIN - 1, npts) and r.dtype.itemsize == 4
        f = netcdf_file(path, "r", mmap=True)
        try:
            def one(i):
                v = f.variables[L.LDASIN[i]]
                s = np.asarray(v[0] if v.dimensions[0] == "Time" else v[:]).reshape(-1)
                assert s.dtype == np.dtype(">f4"), f"{L.LDASIN[i]}: {s.dtype}"
                r[i].view(">f4")[...] = s
            self._map(one, list(range(L.NLDASIN - 1)))
        finally:
            f.close()
        return r

    def file_cosz(self, t: datetime.datetime) -> bool:
        """The input file of t carries COSZ (then it, not the solar geometry, is the step's)."""
        return "COSZ" in self.variables(t)

    def geo(self) -> np.ndarray:
        """(3, n) float64 per column: sin lat, cos lat, lon (radians) -- the
        column factors of timeman.cosz, the same values it evaluates."""
        return np.stack([self._sincos_lat[0], self._sincos_lat[1],
                         np.asarray(self.lon, np.float64)])


# ---- LDASOUT ----------------------------------------------------------------------
def write_ldasout(path: str, grid: Grid, diag: np.ndarray, t: datetime.datetime,
                  cols: np.ndarray | None = None, pool=None):
    """The 16 output fluxes (NMP_O_*, (16, n)) on the grid.  cols: column j of
    diag is land point cols[j] (an engine order; default: land-point order).
    pool: an executor that scatters the fields in parallel."""
    ny, nx = grid.shape
    kind = "f8" if diag.dtype == np.float64 else "f4"
    idx = np.asarray(grid.index) if cols is None else np.asarray(grid.index)[cols]
    # the fields scattered straight into the file's (big-endian) element type
    full = np.empty((len(L.DIAG_OUT), ny * nx), np.dtype(kind).newbyteorder(">"))

    def one(i):
        full[i].fill(FILL)
        full[i][idx] = diag[i]
    if pool is None:
        for i in range(len(L.DIAG_OUT)):
            one(i)
    else:
        for fut in [pool.submit(one, i) for i in range(len(L.DIAG_OUT))]:
            fut.result()
    f = netcdf_file(path, "w")
    try:
        f.createDimension("Time", None)
        f.createDimension("south_north", ny)
        f.createDimension("west_east", nx)
        f.valid_time = t.isoformat()
        dims = ("Time", "south_north", "west_east")
        for i, name in enumerate(L.DIAG_OUT):
            v = f.createVariable(name, kind, dims)
            v._FillValue = np.asarray(FILL, kind)
            v[0] = full[i].reshape(ny, nx)
    finally:
        f.close()


def _nc_name(s: str) -> bytes:
    b = s.encode("latin1")
    return np.array(len(b), ">i4").tobytes() + b + b"\x00" * (-len(b) % 4)


def ldasout_header(grid: Grid, kind: str, t: datetime.datetime) -> bytes:
    """The netCDF-3 classic header write_ldasout's file has (one record of the
    16 flux variables over (Time, south_north, west_east), the valid_time
    global attribute, each variable's _FillValue), built from the format's
    layout: magic, numrecs, dimension / attribute / variable lists, each
    variable's type, per-record size and data offset."""
    ny, nx = grid.shape
    i4 = lambda v: np.array(v, ">i4").tobytes()  # noqa: E731
    item = np.dtype(kind).itemsize
    nc_type = {4: 5, 8: 6}[item]                 # NC_FLOAT, NC_DOUBLE
    fill = np.asarray(FILL, np.dtype(kind).newbyteorder(">")).tobytes()
    h = [b"CDF\x01", i4(1), i4(10), i4(3)]       # NC_DIMENSION, 3 dims
    for name, n in (("Time", 0), ("south_north", ny), ("west_east", nx)):
        h += [_nc_name(name), i4(n)]
    vt = t.isoformat().encode("latin1")
    h += [i4(12), i4(1), _nc_name("valid_time"), i4(2), i4(len(vt)), vt,
          b"\x00" * (-len(vt) % 4)]               # NC_ATTRIBUTE, NC_CHAR
    h += [i4(11), i4(len(L.DIAG_OUT))]           # NC_VARIABLE
    vsize = ny * nx * item
    vsize += -vsize % 4
    metas = []
    for name in L.DIAG_OUT:
        metas.append([_nc_name(name), i4(3), i4(0), i4(1), i4(2), i4(12), i4(1),
                      _nc_name("_FillValue"), i4(nc_type), i4(1), fill, i4(nc_type), i4(vsize)])
    size = sum(len(x) for x in h) + sum(sum(len(x) for x in m) + 4 for m in metas)
    if size + len(metas) * vsize > 2**31 - 1:  # CDF-1 offsets are signed 32-bit
        raise ValueError(f"LDASOUT of {ny} x {nx} {kind} grids exceeds the classic format's "
                         "2 GiB offsets")
    for i, m in enumerate(metas):
        h += m + [i4(size + i * vsize)]         # begin (32-bit offsets, version 1)
    return b"".join(h)


def write_ldasout_grids(path: str, grid: Grid, grids_be: np.ndarray, t: datetime.datetime):
    """An LDASOUT file from the 16 fluxes already on the file's grids in its
    byte order (nmp_ldasout_grid's output: (16, npts) big-endian fp32 or
    fp64, FILL off the land points): the header and the bytes, one write --
    the same file write_ldasout produces from the columns."""
    kind = {4: "f4", 8: "f8"}[grids_be.dtype.itemsize]
    ny, nx = grid.shape
    assert grids_be.shape == (len(L.DIAG_OUT), ny * nx) and grids_be.flags.c_contiguous
    with open(path, "wb") as f:
        f.write(ldasout_header(grid, kind, t))
        f.write(memoryview(grids_be).cast("B"))


def read_ldasout(path: str, grid: Grid) -> np.ndarray:
    raw = read_ldasin(path)
    return np.stack([grid.columns(raw[name]) for name in L.DIAG_OUT])
