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
NFORCING = len(FORCING)
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
