"""ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.

ctypes driver for ``oracle/_ref/libnoahmp_ref.so``: the reference Fortran
(/root/reference/core/*.f90, compiled by oracle/Makefile) behind our batch
harness (oracle/ref_harness.f90).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may use this module, and only as the checker.

The reference keeps tables and options in process-global module variables
(core/module_noahmp_global.f90:17-74, *_param.f90) and `SAVE`d locals
(func.f90:3854-3856), so one process holds one configuration at a time and
must not call it from several threads.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")
LIB_PATH = os.path.join(REF_DIR, "libnoahmp_ref.so")
TBL_DIR = os.path.join(REF_DIR, "tbl")

NST, NSF, NSI, NFC, NDG = 56, 6, 6, 12, 58

# nmp_params float fields in storage order with their element counts
# (== include/noahmp_engine.h struct nmp_params == ref_dump_params order)
PARAM_FLOAT_FIELDS = [
    ("slope", 30), ("csoil", 1), ("zbot", 1), ("czil", 1), ("dkref", 1), ("kdtref", 1),
    ("frzk", 1), ("timean", 1), ("fsatmax", 1), ("mltfct", 1), ("z0sno", 1), ("ssi", 1),
    ("swemax", 1), ("albice", 2), ("alblake", 2), ("omegas", 2), ("betads", 1), ("betais", 1),
    ("emssoil", 1), ("emslake", 1),
    ("bexp", 30), ("smcmax", 30), ("smcref", 30), ("smcwlt", 30), ("psisat", 30), ("dksat", 30),
    ("dwsat", 30), ("quartz", 30), ("kdt", 30), ("frzx", 30), ("albsat", 40), ("albdry", 40),
    ("xl", 27), ("rhol", 54), ("rhos", 54), ("taul", 54), ("taus", 54),
    ("canwmxp", 27), ("dleaf", 27), ("z0mvt", 27), ("hvt", 27), ("hvb", 27), ("den", 27),
    ("rcrown", 27), ("cwpvt", 27), ("sai12m", 324), ("lai12m", 324),
    ("sla", 27), ("dilefc", 27), ("dilefw", 27), ("fragr", 27), ("ltovrc", 27), ("wrrat", 27),
    ("wdpool", 27), ("tdlef", 27), ("rgl", 27), ("hs", 27), ("rsmax", 27), ("rsmin", 27),
    ("topt", 27), ("kc25", 27), ("akc", 27), ("ko25", 27), ("ako", 27), ("vcmx25", 27),
    ("avcmx", 27), ("bp", 27), ("mp", 27), ("qe25", 27), ("aqe", 27), ("folnmx", 27),
    ("tmin", 27), ("rmf25", 27), ("rms25", 27), ("rmr25", 27), ("arm", 27), ("mrp", 27),
    ("slarea", 27), ("eps", 135),
]
PARAM_SHAPES = {"albsat": (20, 2), "albdry": (20, 2), "rhol": (27, 2), "rhos": (27, 2),
                "taul": (27, 2), "taus": (27, 2), "sai12m": (27, 12), "lai12m": (27, 12),
                "eps": (27, 5)}
PARAM_INT_FIELDS = [("nslptyp", 1), ("nsltyp", 1), ("nsoilcol", 1), ("nlutyp", 1),
                    ("isurban", 1), ("iswater", 1), ("isbarren", 1), ("isice", 1),
                    ("isegblf", 1), ("nroot", 27), ("c3c4", 27)]
NPARAM_F = sum(w for _, w in PARAM_FLOAT_FIELDS)
NPARAM_I = sum(w for _, w in PARAM_INT_FIELDS)

_lock = threading.Lock()
_lib = None
_loaded_cfg = None


def available() -> bool:
    return os.path.exists(LIB_PATH) and os.path.exists(os.path.join(TBL_DIR, "GENPARMMP.TBL"))


def _load():
    global _lib
    if _lib is None:
        if not available():
            raise FileNotFoundError(f"reference oracle not built: {LIB_PATH} (run make -C oracle ref)")
        lib = C.CDLL(LIB_PATH)
        f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        lib.ref_set_options.argtypes = [i32p]
        lib.ref_read_tables.argtypes = [C.c_char_p, C.c_int32, C.c_char_p, C.c_int32]
        lib.ref_dump_params.argtypes = [f32p, C.c_int32, i32p, C.c_int32]
        lib.ref_sflx_batch.argtypes = [C.c_int32, C.c_float, C.c_int32, C.c_float, f32p,
                                       f32p, i32p, f32p, i32p, f32p, f32p, i32p]
        if hasattr(lib, "ref_frh2o"):
            lib.ref_frh2o.argtypes = [C.c_int32, i32p, f32p, f32p, f32p, f32p, i32p]
        if hasattr(lib, "ref_calhum"):
            lib.ref_calhum.argtypes = [C.c_int32, f32p, f32p, f32p, f32p]
        if hasattr(lib, "ref_set_ficeold"):
            lib.ref_set_ficeold.argtypes = [C.c_void_p, C.c_int32]
        if hasattr(lib, "ref_sflx_run"):
            lib.ref_sflx_run.argtypes = [C.c_int32, C.c_int32, C.c_float, C.c_int32, C.c_float,
                                         f32p, f32p, i32p, f32p, i32p, f32p, C.c_int32, f32p, i32p]
        _lib = lib
    return _lib


def configure(options: tuple, soil_tag: str = "STAS", veg_tag: str = "USGS"):
    """Read the tables (from oracle/_ref/tbl, the reference reads the CWD) and set options."""
    global _loaded_cfg
    lib = _load()
    with _lock:
        if _loaded_cfg != (soil_tag, veg_tag):
            cwd = os.getcwd()
            os.chdir(TBL_DIR)
            try:
                lib.ref_read_tables(soil_tag.encode(), len(soil_tag), veg_tag.encode(), len(veg_tag))
            finally:
                os.chdir(cwd)
            _loaded_cfg = (soil_tag, veg_tag)
        lib.ref_set_options(np.asarray(options, np.int32))


def dump_params() -> dict:
    """Every table value as read by the reference readers (after configure())."""
    lib = _load()
    fb = np.zeros(NPARAM_F, np.float32)
    ib = np.zeros(NPARAM_I + 1, np.int32)
    lib.ref_dump_params(fb, NPARAM_F, ib, NPARAM_I + 1)
    assert ib[-1] == NPARAM_F, (ib[-1], NPARAM_F)
    out, k = {}, 0
    for name, w in PARAM_FLOAT_FIELDS:
        a = fb[k:k + w].copy()
        out[name] = a.reshape(PARAM_SHAPES[name]) if name in PARAM_SHAPES else (a if w > 1 else a[0])
        k += w
    k = 0
    for name, w in PARAM_INT_FIELDS:
        a = ib[k:k + w].copy()
        out[name] = a if w > 1 else int(a[0])
        k += w
    return out


def step(zsoil, dt, yearlen, julian, state, isnow, static_f, static_i, forcing, ficeold=None):
    """One reference noahmp_sflx step for every column.

    SoA inputs (nfield, n) like the engine; returns (state', isnow', diag(58,n), status).
    ficeold (3, n): noahmp_sflx's FICEOLD argument per column (default: the
    step-start ice fraction of the active snow layers, 0 elsewhere)."""
    lib = _load()
    n = isnow.shape[0]
    st = np.array(np.asarray(state, np.float32).T, order="C")  # a copy: written in place
    isn = np.ascontiguousarray(isnow, np.int32).copy()
    sf = np.ascontiguousarray(np.asarray(static_f, np.float32).T)
    si = np.ascontiguousarray(np.asarray(static_i, np.int32).T)
    fc = np.ascontiguousarray(np.asarray(forcing, np.float32).T)
    dg = np.zeros((n, NDG), np.float32)
    status = np.zeros(n, np.int32)
    fo = None if ficeold is None else np.ascontiguousarray(np.asarray(ficeold, np.float32).T)
    with _lock:
        if fo is not None:
            lib.ref_set_ficeold(fo.ctypes.data, n)
        try:
            lib.ref_sflx_batch(n, float(dt), int(yearlen), float(julian),
                               np.ascontiguousarray(zsoil, np.float32), st, isn, sf, si, fc, dg,
                               status)
        finally:
            if fo is not None:
                lib.ref_set_ficeold(None, 0)
    return st.T.copy(), isn, dg.T.copy(), status


class Records:
    """Column records in the harness layout (one column's fields contiguous),
    transposed once, so a timed loop can call `run` without host transposes."""

    def __init__(self, state, isnow, static_f, static_i, forcings):
        self.st = np.array(np.asarray(state, np.float32).T, order="C")  # a copy: written in place
        self.isn = np.ascontiguousarray(isnow, np.int32).copy()
        self.sf = np.ascontiguousarray(np.asarray(static_f, np.float32).T)
        self.si = np.ascontiguousarray(np.asarray(static_i, np.int32).T)
        self.fc = np.ascontiguousarray(np.asarray(forcings, np.float32).transpose(0, 2, 1))
        n = self.isn.shape[0]
        self.dg = np.zeros((n, NDG), np.float32)
        self.status = np.zeros(n, np.int32)


def run(zsoil, dt, yearlen, julian0, rec: Records, nsteps: int):
    """nsteps reference steps of `rec` in place (ref_sflx_run: the time loop in
    the Fortran harness, forcing cycled over rec.fc's period)."""
    lib = _load()
    with _lock:
        lib.ref_sflx_run(rec.isn.shape[0], int(nsteps), float(dt), int(yearlen), float(julian0),
                         np.ascontiguousarray(zsoil, np.float32), rec.st, rec.isn, rec.sf, rec.si,
                         rec.fc, rec.fc.shape[0], rec.dg, rec.status)
    return rec


def frh2o(sltyp, tk, smc, sh2o):
    """The reference's public frh2o (func.f90:4494-4598) over arrays (after
    configure()): (free water, status bits)."""
    lib = _load()
    n = len(tk)
    out = np.zeros(n, np.float32)
    st = np.zeros(n, np.int32)
    with _lock:
        lib.ref_frh2o(n, np.ascontiguousarray(sltyp, np.int32), np.ascontiguousarray(tk, np.float32),
                      np.ascontiguousarray(smc, np.float32), np.ascontiguousarray(sh2o, np.float32),
                      out, st)
    return out, st


def calhum(sfctmp, sfcprs):
    """The reference's calhum (func.f90:3958-3984) over arrays: (Q2SAT, DQSDT2)."""
    lib = _load()
    n = len(sfctmp)
    q = np.zeros(n, np.float32)
    d = np.zeros(n, np.float32)
    with _lock:
        lib.ref_calhum(n, np.ascontiguousarray(sfctmp, np.float32),
                       np.ascontiguousarray(sfcprs, np.float32), q, d)
    return q, d
