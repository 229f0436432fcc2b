"""ctypes binding of libnoahmp_engine.so (include/noahmp_engine.h).

The HIP library is the only compute path: if it is missing this module raises
instead of falling back to anything else.
"""
from __future__ import annotations

import ctypes as C
import os

from . import build as _build

NMP_OPTION_FIELDS = ["opt_veg", "opt_crs", "opt_btr", "opt_run", "opt_sfc", "opt_frz",
                     "opt_inf", "opt_rad", "opt_alb", "opt_snf", "opt_tbot", "opt_stc"]


class NmpOptions(C.Structure):
    _fields_ = [(n, C.c_int32) for n in NMP_OPTION_FIELDS]


# struct nmp_params, field order of the header
_F = C.c_float
_I = C.c_int32
_PARAM_LAYOUT = [
    ("slope", _F * 30), ("csoil", _F), ("zbot", _F), ("czil", _F), ("dkref", _F), ("kdtref", _F),
    ("frzk", _F), ("timean", _F), ("fsatmax", _F), ("mltfct", _F), ("z0sno", _F), ("ssi", _F),
    ("swemax", _F), ("albice", _F * 2), ("alblake", _F * 2), ("omegas", _F * 2),
    ("betads", _F), ("betais", _F), ("emssoil", _F), ("emslake", _F),
    ("bexp", _F * 30), ("smcmax", _F * 30), ("smcref", _F * 30), ("smcwlt", _F * 30),
    ("psisat", _F * 30), ("dksat", _F * 30), ("dwsat", _F * 30), ("quartz", _F * 30),
    ("kdt", _F * 30), ("frzx", _F * 30), ("albsat", (_F * 2) * 20), ("albdry", (_F * 2) * 20),
    ("xl", _F * 27), ("rhol", (_F * 2) * 27), ("rhos", (_F * 2) * 27), ("taul", (_F * 2) * 27),
    ("taus", (_F * 2) * 27), ("canwmxp", _F * 27), ("dleaf", _F * 27), ("z0mvt", _F * 27),
    ("hvt", _F * 27), ("hvb", _F * 27), ("den", _F * 27), ("rcrown", _F * 27), ("cwpvt", _F * 27),
    ("sai12m", (_F * 12) * 27), ("lai12m", (_F * 12) * 27),
    ("sla", _F * 27), ("dilefc", _F * 27), ("dilefw", _F * 27), ("fragr", _F * 27),
    ("ltovrc", _F * 27), ("wrrat", _F * 27), ("wdpool", _F * 27), ("tdlef", _F * 27),
    ("rgl", _F * 27), ("hs", _F * 27), ("rsmax", _F * 27), ("rsmin", _F * 27), ("topt", _F * 27),
    ("kc25", _F * 27), ("akc", _F * 27), ("ko25", _F * 27), ("ako", _F * 27), ("vcmx25", _F * 27),
    ("avcmx", _F * 27), ("bp", _F * 27), ("mp", _F * 27), ("qe25", _F * 27), ("aqe", _F * 27),
    ("folnmx", _F * 27), ("tmin", _F * 27), ("rmf25", _F * 27), ("rms25", _F * 27),
    ("rmr25", _F * 27), ("arm", _F * 27), ("mrp", _F * 27), ("slarea", _F * 27),
    ("eps", (_F * 5) * 27),
    ("nslptyp", _I), ("nsltyp", _I), ("nsoilcol", _I), ("nlutyp", _I), ("isurban", _I),
    ("iswater", _I), ("isbarren", _I), ("isice", _I), ("isegblf", _I),
    ("nroot", _I * 27), ("c3c4", _I * 27),
]


class NmpParams(C.Structure):
    _fields_ = _PARAM_LAYOUT


PARAM_FIELDS = [n for n, _ in _PARAM_LAYOUT]

_lib = None


def library_path() -> str:
    return _build.LIB_PATH


def load(build_if_missing: bool = False):
    """Load the engine library (building it first only when asked)."""
    global _lib
    if _lib is not None:
        return _lib
    path = _build.LIB_PATH
    if not os.path.exists(path):
        if build_if_missing:
            _build.build()
        else:
            raise RuntimeError(
                f"noahmp engine library not built ({path}); run __graft_entry__.build() "
                "or python noahmp-1_amd/build.py -- there is no CPU fallback")
    if path == _build.DEFAULT_LIB_PATH or os.environ.get("NOAHMP_CHECK_HASH") == "1":
        # the library must come from the sources beside it (a stale .so that
        # travelled with the snapshot would otherwise run silently)
        got, want = _build.built_hash(path), _build.source_hash()
        if got != want:
            if build_if_missing:
                _build.build()
            else:
                raise RuntimeError(
                    f"stale noahmp engine library {path}: built from sources {got}, the sources "
                    f"here hash to {want}; rebuild with __graft_entry__.build()")
    lib = C.CDLL(path)
    vp, i32p, f32p = C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_float)
    lib.nmp_read_tables.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(NmpParams)]
    lib.nmp_init.argtypes = [C.POINTER(NmpParams), C.POINTER(NmpOptions), C.c_int, C.c_int,
                             C.POINTER(vp)]
    lib.nmp_set_math.argtypes = [vp, C.c_int]
    lib.nmp_set_cols_per_wave.argtypes = [vp, C.c_int]
    lib.nmp_step.argtypes = [vp, C.c_int64, C.c_int64, f32p, C.c_float, C.c_float, C.c_int32,
                             vp, vp, vp, vp, vp, vp, C.c_int, vp, vp]
    lib.nmp_step_binned.argtypes = [vp, C.c_int64, C.c_int64, f32p, C.c_float, C.c_float,
                                     C.c_int32, vp, vp, vp, vp, vp, vp, C.c_int, vp, vp, vp, vp]
    lib.nmp_rebin.argtypes = [vp, C.c_int64, vp, vp, C.c_int32, vp]
    lib.nmp_forcing_synth.argtypes = [vp, C.c_int64, C.c_int64, vp, C.c_double, C.c_int32,
                                      C.c_uint64, C.c_int64, C.c_int64, vp, vp]
    lib.nmp_forcing_from_ldasin.argtypes = [vp, C.c_int64, C.c_int64, vp, vp, vp]
    lib.nmp_forcing_from_ldasin_geo.argtypes = [vp, C.c_int64, C.c_int64, vp, vp, C.c_double,
                                                C.c_double, C.c_double, vp, vp]
    lib.nmp_ldasin_ingest.argtypes = [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp, vp]
    lib.nmp_ldasout_grid.argtypes = [vp, C.c_int64, C.c_int64, C.c_int64, C.c_int, vp, vp,
                                     C.c_double, vp, vp]
    lib.nmp_run.argtypes = [vp, C.c_int64, C.c_int64, f32p, C.c_float, C.c_float, C.c_int32,
                            C.c_int32, vp, vp, vp, vp, vp, C.c_int64, C.c_int32, vp, C.c_int, vp,
                            vp]
    if hasattr(lib, "nmp_run_out"):  # (absent from ABI-1 builds timed by tools/sweep.sh)
        lib.nmp_run_out.argtypes = [vp, C.c_int64, C.c_int64, f32p, C.c_float, C.c_float,
                                    C.c_int32, C.c_int32, vp, vp, vp, vp, vp, C.c_int64,
                                    C.c_int32, vp, C.c_int, C.c_int32, C.c_int32, C.c_int64, vp,
                                    vp]
    lib.nmp_state_from_aos.argtypes = [vp, C.c_int64, C.c_int64, vp, vp, vp]
    lib.nmp_sflx_columns.argtypes = [vp, vp, C.c_int64]
    lib.nmp_sflx_column.argtypes = [vp, vp]
    lib.nmp_option_set.argtypes = [vp, C.c_int]
    lib.nmp_set_launch_variant.argtypes = [vp, C.c_int]
    lib.nmp_type_size.argtypes = [C.c_int]
    lib.nmp_type_size.restype = C.c_int64
    lib.nmp_frh2o.argtypes = [vp, C.c_int64, vp, vp, vp, vp, vp, vp, vp]
    lib.nmp_frh2o_host.argtypes = [vp, C.c_int64, vp, vp, vp, vp, vp, vp]
    lib.nmp_calhum.argtypes = [vp, C.c_int64, vp, vp, vp, vp, vp]
    lib.nmp_calhum_host.argtypes = [vp, C.c_int64, vp, vp, vp, vp]
    lib.nmp_engine_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    C.POINTER(NmpOptions)]
    lib.nmp_finalize.argtypes = [vp]
    lib.nmp_finalize.restype = None
    lib.nmp_strerror.argtypes = [C.c_int]
    lib.nmp_strerror.restype = C.c_char_p
    lib.nmp_abi_version.restype = C.c_int
    lib.nmp_build_hash.restype = C.c_char_p
    _lib = lib
    return lib


EXPORTED_SYMBOLS = ["nmp_read_tables", "nmp_init", "nmp_step", "nmp_step_binned", "nmp_rebin", "nmp_forcing_synth", "nmp_forcing_from_ldasin", "nmp_forcing_from_ldasin_geo", "nmp_ldasin_ingest", "nmp_ldasout_grid",
                    "nmp_run", "nmp_run_out", "nmp_frh2o", "nmp_frh2o_host", "nmp_calhum",
                    "nmp_calhum_host",
                    "nmp_state_from_aos", "nmp_sflx_columns", "nmp_sflx_column",
                    "nmp_engine_info", "nmp_option_set", "nmp_set_launch_variant", "nmp_type_size", "nmp_set_math", "nmp_set_cols_per_wave", "nmp_finalize", "nmp_strerror",
                    "nmp_abi_version", "nmp_build_hash"]


class NmpError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        lib = load()
        msg = lib.nmp_strerror(code).decode()
        super().__init__(f"{what}: {msg} (code {code})" if what else f"{msg} (code {code})")
        self.code = code


def check(code: int, what: str = ""):
    if code != 0:
        raise NmpError(code, what)
