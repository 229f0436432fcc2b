"""Field layouts of the engine's SoA buffers.

Mirrors the enums of ``include/noahmp_engine.h`` (tests/test_layout.py checks
that every offset here equals the header's).  The per-column variable set is
the argument list of the reference ``noahmp_sflx``
(/root/reference/core/module_noahmp_func.f90:66-91); the 7-entry snow/soil
arrays use C index k for Fortran layer k-2 (``-NSNOW+1:NSOIL``).
"""
from __future__ import annotations

NSOIL = 4
NSNOW = 3
NLAYER = 7

# (name, width) in storage order -- NMP_S_*
STATE_FIELDS = [
    ("STC", 7), ("ZSNSO", 7), ("SNICE", 3), ("SNLIQ", 3), ("SH2O", 4), ("SMC", 4),
    ("TV", 1), ("TG", 1), ("TAH", 1), ("EAH", 1), ("FWET", 1), ("CANLIQ", 1),
    ("CANICE", 1), ("QSFC", 1), ("SNOWH", 1), ("SNEQV", 1), ("SNEQVO", 1), ("ALBOLD", 1),
    ("TAUSS", 1), ("QSNOW", 1), ("ZWT", 1), ("WA", 1), ("WT", 1), ("WSLAKE", 1),
    ("LAI", 1), ("SAI", 1), ("LFMASS", 1), ("RTMASS", 1), ("STMASS", 1), ("WOOD", 1),
    ("STBLCP", 1), ("FASTCP", 1), ("CM", 1), ("CH", 1),
]
STATIC_F = ["LAT", "ZLVL", "SHDFAC", "SHDMAX", "TBOT", "FOLN"]
STATIC_I = ["VEGTYP", "SOILTYP", "SLOPETYP", "SOILCOLOR", "IST", "ICE"]
FORCING = ["SFCTMP", "SFCPRS", "PSFC", "UU", "VV", "Q2", "SOLDN", "LWDN", "PRCP", "COSZ",
           "CO2AIR", "O2AIR"]
DIAG_FULL = [
    "FSA", "FSR", "FIRA", "FSH", "SSOIL", "FCEV", "FGEV", "FCTR", "ECAN", "ETRAN", "EDIR", "TRAD",
    "TGB", "TGV", "T2MV", "T2MB", "Q2V", "Q2B", "RUNSRF", "RUNSUB", "APAR", "PSN", "SAV", "SAG",
    "FSNO", "NEE", "GPP", "NPP", "FVEG", "ALBEDO", "QSNBOT", "PONDING", "PONDING1", "PONDING2",
    "RSSUN", "RSSHA", "BGAP", "WGAP", "CHV", "CHB", "EMISSI", "SHG", "SHC", "SHB", "EVG", "EVB",
    "GHV", "GHB", "IRG", "IRC", "IRB", "TR", "EVC", "CHLEAF", "CHUC", "CHV2", "CHB2", "FPICE",
]
DIAG_OUT = ["FSA", "FSR", "FIRA", "FSH", "SSOIL", "FCEV", "FGEV", "FCTR", "ECAN", "ETRAN", "EDIR",
            "TRAD", "RUNSRF", "RUNSUB", "T2M", "ALBEDO"]

# status bits (NMP_ST_*)
ST_ERRSW, ST_ERRENG, ST_FIRE, ST_HCAN, ST_ZLVL, ST_FLERCH, ST_OPTVEG, ST_STOP = (
    1, 2, 4, 8, 16, 32, 64, 128)

DIAG_NONE, DIAG_OUT_LEVEL, DIAG_FULL_LEVEL = 0, 1, 2

OPTION_NAMES = ["opt_veg", "opt_crs", "opt_btr", "opt_run", "opt_sfc", "opt_frz",
                "opt_inf", "opt_rad", "opt_alb", "opt_snf", "opt_tbot", "opt_stc"]
# case.nml options (run/case.nml:29-37) + the SURVEY 5 defaults for the five
# options the namelist lacks (opt_crs, opt_sfc, opt_frz, opt_alb, opt_stc).
CASE_NML_OPTIONS = dict(opt_veg=1, opt_crs=1, opt_btr=1, opt_run=1, opt_sfc=1, opt_frz=1,
                        opt_inf=1, opt_rad=1, opt_alb=2, opt_snf=1, opt_tbot=1, opt_stc=1)
# valid ranges (core/module_noahmp_global.f90:17-74)
OPTION_RANGES = dict(opt_veg=(1, 5), opt_crs=(1, 2), opt_btr=(1, 3), opt_run=(1, 4),
                     opt_sfc=(1, 2), opt_frz=(1, 2), opt_inf=(1, 2), opt_rad=(1, 3),
                     opt_alb=(1, 2), opt_snf=(1, 3), opt_tbot=(1, 2), opt_stc=(1, 2))


# struct nmp_sflx_args: the 131 noahmp_sflx dummy arguments in dummy order
# (core/module_noahmp_func.f90:66-91) + the status word; (name, "i"|"f", count)
SFLX_ARGS = (
    [("iloc", "i", 1), ("jloc", "i", 1), ("lat", "f", 1), ("yearlen", "i", 1),
     ("julian", "f", 1), ("cosz", "f", 1), ("dt", "f", 1), ("dx", "f", 1), ("dz8w", "f", 1),
     ("nsoil", "i", 1), ("zsoil", "f", NSOIL), ("nsnow", "i", 1), ("shdfac", "f", 1),
     ("shdmax", "f", 1)]
    + [(n, "i", 1) for n in ("slptyp", "sltyp", "lutyp", "ice", "ist", "isc", "iz0tlnd")]
    + [(n, "f", 1) for n in ("sfctmp", "sfcprs", "psfc", "uu", "vv", "q2", "qc", "soldn", "lwdn",
                             "prcp", "tbot", "co2air", "o2air", "foln")]
    + [("ficeold", "f", NSNOW), ("pblh", "f", 1), ("zlvl", "f", 1), ("albold", "f", 1),
       ("sneqvo", "f", 1), ("stc", "f", NLAYER), ("soilwat", "f", NSOIL), ("smc", "f", NSOIL)]
    + [(n, "f", 1) for n in ("tah", "eah", "fwet", "canliq", "canice", "tv", "tg", "qsfc",
                             "qsnow")]
    + [("isnow", "i", 1), ("zsnso", "f", NLAYER), ("snowh", "f", 1), ("sneqv", "f", 1),
       ("snice", "f", NSNOW), ("snliq", "f", NSNOW)]
    + [(n, "f", 1) for n in ("zwt", "wa", "wt", "wslake", "lfmass", "rtmass", "stmass", "wood",
                             "stblcp", "fastcp", "lai", "sai", "cm", "ch", "tauss")]
    + [("out", "f", 58), ("status", "i", 1)]
)


def sflx_args_dtype():
    """numpy structured dtype with the byte layout of struct nmp_sflx_args."""
    import numpy as np
    return np.dtype([(n, np.int32 if k == "i" else np.float32) if w == 1 else
                     (n, np.int32 if k == "i" else np.float32, (w,)) for n, k, w in SFLX_ARGS])


_REC_STATE = {"SH2O": "soilwat"}
_REC_STATIC_I = {"VEGTYP": "lutyp", "SOILTYP": "sltyp", "SLOPETYP": "slptyp",
                 "SOILCOLOR": "isc", "IST": "ist", "ICE": "ice"}


def sflx_records(state, isnow, static_f, static_i, forcing, zsoil, dt, julian, yearlen):
    """nmp_sflx_args records (host) from field-major SoA arrays (n columns):
    the reference calling sequence of the same step, FICEOLD derived from
    SNICE/SNLIQ as the offline and WRF drivers do."""
    import numpy as np
    n = int(np.shape(isnow)[0])
    r = np.zeros(n, sflx_args_dtype())
    r["nsoil"], r["nsnow"], r["yearlen"] = NSOIL, NSNOW, int(yearlen)
    r["dt"], r["julian"] = np.float32(dt), np.float32(julian)
    r["zsoil"] = np.asarray(zsoil, np.float32)[None, :]
    for name, w in STATE_FIELDS:
        o = STATE_OFF[name][0]
        key = _REC_STATE.get(name, name.lower())
        r[key] = state[o:o + w].T if w > 1 else state[o]
    r["isnow"] = isnow
    for i, name in enumerate(STATIC_F):
        r[name.lower()] = static_f[i]
    for i, name in enumerate(STATIC_I):
        r[_REC_STATIC_I[name]] = static_i[i]
    for i, name in enumerate(FORCING):
        r[name.lower()] = forcing[i]
    with np.errstate(invalid="ignore", divide="ignore"):
        act = np.arange(NSNOW)[None, :] >= (np.asarray(isnow)[:, None] + NSNOW)
        fo = r["snice"] / (r["snice"] + r["snliq"])
    r["ficeold"] = np.where(act, fo, np.float32(0.0))
    return r


def soa_from_records(r):
    """(state (56, n), isnow (n,), diag (58, n), status (n,)) of records after a call."""
    import numpy as np
    n = r.shape[0]
    st = np.empty((NSTATE, n), np.float32)
    for name, w in STATE_FIELDS:
        o = STATE_OFF[name][0]
        v = r[_REC_STATE.get(name, name.lower())]
        st[o:o + w] = v.T if w > 1 else v
    return st, r["isnow"].copy(), np.ascontiguousarray(r["out"].T), r["status"].copy()


def _offsets(fields):
    off, out = 0, {}
    for name, w in fields:
        out[name] = (off, w)
        off += w
    return out, off


STATE_OFF, NSTATE = _offsets(STATE_FIELDS)
assert NSTATE == 56
NSTATIC_F = len(STATIC_F)
NSTATIC_I = len(STATIC_I)
# LDASIN block of nmp_forcing_from_ldasin (NMP_L_*): the 8 variables of an
# LDASIN file (ncio.py) plus the step's COSZ, fp32
LDASIN = ["T2D", "Q2D", "U2D", "V2D", "PSFC", "RAINRATE", "SWDOWN", "LWDOWN", "COSZ"]
NLDASIN = len(LDASIN)
NFORCING = len(FORCING)
# climate record of the device forcing generator (NMP_CLIM_*, nmp_forcing_synth)
CLIMATE = ["LAT", "LON", "T0", "AMP", "RH", "PRES", "WIND_U", "WIND_V", "WET"]
NCLIM = len(CLIMATE)
NDIAG_FULL = len(DIAG_FULL)
NDIAG_OUT = len(DIAG_OUT)
assert NDIAG_FULL == 58 and NDIAG_OUT == 16


def s(name):
    """Slice of a state field along the field axis."""
    o, w = STATE_OFF[name]
    return slice(o, o + w)


def si(name):
    return STATE_OFF[name][0]


def options_tuple(opts: dict) -> tuple:
    return tuple(int(opts[k]) for k in OPTION_NAMES)
