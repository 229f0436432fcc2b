"""ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.

ctypes driver for the plain-C restatement (oracle/noahmp_oracle.c), built as
build/liboracle_f32.so and build/liboracle_f64.so by oracle/Makefile.
Same SoA interface as oracle/ref.py.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ref import PARAM_FLOAT_FIELDS, PARAM_INT_FIELDS, PARAM_SHAPES, NPARAM_F, NPARAM_I

HERE = os.path.dirname(os.path.abspath(__file__))
LIBS = {4: os.path.join(HERE, "build", "liboracle_f32.so"),
        8: os.path.join(HERE, "build", "liboracle_f64.so"),
        "cr": os.path.join(HERE, "build", "liboracle_f32cr.so"),
        "4s": os.path.join(HERE, "build", "liboracle_f32_stats.so"),
        "8s": os.path.join(HERE, "build", "liboracle_f64_stats.so"),
        "4d": os.path.join(HERE, "build", "liboracle_f32_divstats.so")}
# trip counts recorded by the stats builds, per column (noahmp_oracle.c ITER_STAT)
STAT_LOOPS = ("vege_flux Newton", "stomata bisection", "frh2o", "soilwater sub-steps",
              "bare_flux Newton")
NST, NSF, NSI, NFC, NDG = 56, 6, 6, 12, 58
_libs = {}


def available(precision: int = 4) -> bool:
    return os.path.exists(LIBS[precision])


def pack_params(P: dict) -> bytes:
    """dict (ref.dump_params() layout) -> bytes of `struct nmp_params`."""
    fl = []
    for name, w in PARAM_FLOAT_FIELDS:
        a = np.asarray(P[name], np.float32).reshape(-1)
        assert a.size == w, (name, a.size, w)
        fl.append(a)
    il = []
    for name, w in PARAM_INT_FIELDS:
        a = np.asarray(P[name], np.int32).reshape(-1)
        assert a.size == w, (name, a.size, w)
        il.append(a)
    return np.concatenate(fl).tobytes() + np.concatenate(il).tobytes()


def _lib(precision):
    if precision not in _libs:
        if not available(precision):
            raise FileNotFoundError(f"{LIBS[precision]} missing (run make -C oracle port)")
        lib = C.CDLL(LIBS[precision])
        rt = np.float64 if precision in (8, "8s") else np.float32
        rp = np.ctypeslib.ndpointer(rt, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        creal = C.c_double if precision in (8, "8s") else C.c_float
        lib.oracle_sflx_batch.argtypes = [C.c_int32, creal, C.c_int32, creal, rp, rp, ip, rp, ip,
                                          rp, rp, ip, C.c_char_p, C.c_void_p]
        lib.oracle_sflx_run.argtypes = [C.c_int32, C.c_int32, creal, C.c_int32, creal, rp, rp, ip,
                                        rp, ip, rp, C.c_int32, rp, ip, C.c_char_p, C.c_void_p]
        assert lib.oracle_real_bytes() == (8 if precision in (8, "8s") else 4)
        if precision in ("4s", "8s"):
            lib.oracle_set_stats.argtypes = [C.c_void_p]
        if precision == "4d":
            lib.oracle_div_stats.argtypes = [C.c_void_p, C.c_int]
        _libs[precision] = (lib, rt)
    return _libs[precision]


def step(P: dict, options, zsoil, dt, yearlen, julian, state, isnow, static_f, static_i, forcing,
         precision=4):
    """One step of the C restatement.  SoA in, SoA out: (state', isnow', diag(58,n), status).

    precision: 4 (bit-exact to the reference), 8 (fp64), or "cr" (fp32 with
    correctly rounded libm -- what the engine's default math computes)."""
    lib, rt = _lib(precision)
    n = isnow.shape[0]
    st = np.array(np.asarray(state, rt).T, order="C")  # a copy: written in place
    isn = np.ascontiguousarray(isnow, np.int32).copy()
    sf = np.ascontiguousarray(np.asarray(static_f, rt).T)
    si = np.ascontiguousarray(np.asarray(static_i, np.int32).T)
    fc = np.ascontiguousarray(np.asarray(forcing, rt).T)
    dg = np.zeros((n, NDG), rt)
    status = np.zeros(n, np.int32)
    opts = (C.c_int32 * 12)(*[int(x) for x in options])
    lib.oracle_sflx_batch(n, dt, int(yearlen), julian, np.ascontiguousarray(zsoil, rt), st, isn, sf,
                          si, fc, dg, status, pack_params(P), C.addressof(opts))
    return st.T.copy(), isn, dg.T.copy(), status


def step_stats(P: dict, options, zsoil, dt, yearlen, julian, state, isnow, static_f, static_i,
               forcing, precision=4):
    """step() through the trip-count build of `precision` (4 or 8): returns
    step()'s tuple plus an (n, 5) int32 array of loop trip counts (STAT_LOOPS)."""
    key = {4: "4s", 8: "8s"}[precision]
    lib, _ = _lib(key)
    n = isnow.shape[0]
    buf = np.zeros((n, 8), np.int32)
    lib.oracle_set_stats(buf.ctypes.data)
    try:
        out = step(P, options, zsoil, dt, yearlen, julian, state, isnow, static_f, static_i,
                   forcing, precision=key)
    finally:
        lib.oracle_set_stats(None)
    return (*out, buf[:, :len(STAT_LOOPS)].copy())


def div_stats(reset: bool = False) -> np.ndarray:
    """Division operand ranges recorded by the "4d" build since the last reset
    (noahmp_oracle.c ORACLE_DIV_STATS): (40 sites, 8) = min|a|, max|a|, min|b|,
    max|b|, min|q|, max|q| over nonzero finite values, calls, zero numerators."""
    lib, _ = _lib("4d")
    out = np.zeros((40, 8), np.float64)
    lib.oracle_div_stats(out.ctypes.data, int(reset))
    return out


def prepare_run(P: dict, options, zsoil, dt, yearlen, julian0, state, isnow, static_f, static_i,
                forcings, nsteps: int, precision: int = 4):
    """run() split in two: the host transposes happen here, the returned
    callable is only the library's time loop (the CPU baseline times that) and
    returns (state', isnow', diag, status) of the last step."""
    lib, rt = _lib(precision)
    n = isnow.shape[0]
    st = np.array(np.asarray(state, rt).T, order="C")  # a copy: written in place
    isn = np.ascontiguousarray(isnow, np.int32).copy()
    sf = np.ascontiguousarray(np.asarray(static_f, rt).T)
    si = np.ascontiguousarray(np.asarray(static_i, np.int32).T)
    fc = np.ascontiguousarray(np.asarray(forcings, rt).transpose(0, 2, 1))
    dg = np.zeros((n, NDG), rt)
    status = np.zeros(n, np.int32)
    opts = (C.c_int32 * 12)(*[int(x) for x in options])
    zs = np.ascontiguousarray(zsoil, rt)
    packed = pack_params(P)

    def go():
        lib.oracle_sflx_run(n, nsteps, dt, int(yearlen), julian0, zs, st, isn, sf, si, fc,
                            fc.shape[0], dg, status, packed, C.addressof(opts))
        return st.T.copy(), isn, dg.T.copy(), status
    return go


def run(P: dict, options, zsoil, dt, yearlen, julian0, state, isnow, static_f, static_i,
        forcings, nsteps: int, precision: int = 4):
    """nsteps steps over a forcing cycle forcings[(period, 12, n)]."""
    return prepare_run(P, options, zsoil, dt, yearlen, julian0, state, isnow, static_f, static_i,
                       forcings, nsteps, precision)()


# ---- single routines (the code sflx_column calls), fp32 bit-exact build ----
def _rt(name, *argtypes, precision: int = 4):
    lib, _ = _lib(precision)
    f = getattr(lib, name)
    f.argtypes = list(argtypes)
    f.restype = None
    return f


def esat(t):
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    t = np.ascontiguousarray(t, np.float32)
    out = np.zeros((t.size, 4), np.float32)
    _rt("oracle_esat", C.c_int32, f32p, f32p)(t.size, t, out)
    return out


def tdfcnd(P: dict, sltyp, smc, sh2o):
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
    n = len(smc)
    out = np.zeros(n, np.float32)
    _rt("oracle_tdfcnd", C.c_char_p, C.c_int32, i32p, f32p, f32p, f32p)(
        pack_params(P), n, np.ascontiguousarray(sltyp, np.int32),
        np.ascontiguousarray(smc, np.float32), np.ascontiguousarray(sh2o, np.float32), out)
    return out


def frh2o(P: dict, sltyp, tk, smc, sh2o, precision: int = 4):
    rt = np.float32 if precision == 4 else np.float64
    rp = np.ctypeslib.ndpointer(rt, flags="C_CONTIGUOUS")
    i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
    n = len(tk)
    out = np.zeros(n, rt)
    st = np.zeros(n, np.int32)
    _rt("oracle_frh2o", C.c_char_p, C.c_int32, i32p, rp, rp, rp, rp, i32p, precision=precision)(
        pack_params(P), n, np.ascontiguousarray(sltyp, np.int32), np.ascontiguousarray(tk, rt),
        np.ascontiguousarray(smc, rt), np.ascontiguousarray(sh2o, rt), out, st)
    return out, st


def calhum(sfctmp, sfcprs, precision: int = 4):
    """calhum (func.f90:3958-3984) over arrays: (Q2SAT, DQSDT2)."""
    rt = np.float32 if precision == 4 else np.float64
    rp = np.ctypeslib.ndpointer(rt, flags="C_CONTIGUOUS")
    n = len(sfctmp)
    q, d = np.zeros(n, rt), np.zeros(n, rt)
    _rt("oracle_calhum", C.c_int32, rp, rp, rp, rp, precision=precision)(
        n, np.ascontiguousarray(sfctmp, rt), np.ascontiguousarray(sfcprs, rt), q, d)
    return q, d


def rosr12(kt, a, b, c, d):
    """(n, 7) systems solved on layers kt..6: returns (p, c', delta)."""
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
    n = len(kt)
    c = np.array(c, np.float32, order="C")
    p = np.zeros((n, 7), np.float32)
    dl = np.zeros((n, 7), np.float32)
    _rt("oracle_rosr12", C.c_int32, i32p, f32p, f32p, f32p, f32p, f32p, f32p)(
        n, np.ascontiguousarray(kt, np.int32), np.ascontiguousarray(a, np.float32),
        np.ascontiguousarray(b, np.float32), c, np.ascontiguousarray(d, np.float32), p, dl)
    return p, c, dl
