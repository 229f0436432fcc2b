"""Mid-loop fallback probe (run by tests/test_gpu_parity.py in a child process).

The probe library (`lib_probe_midloop.so`, built by __graft_entry__.build()
from the shipped sources with the per-iteration windows narrowed:
NMP_DOM_TV_HI / NMP_DOM_TGB_HI / NMP_DOM_RAHG_HI, and the numerator windows of
CTR / TR / DTV / DTG raised to |x| >= 4 (NMP_DOM_NUM_LO_EXP=2), plus
NMP_COUNT_FALLBACK)
sends many lanes out of the range proof's domain PART WAY through the canopy
and bare Newton loops, after the fast loop has changed TV/TAH/EAH, QSFC and
the first iteration's stomata outputs.  Those lanes re-run the loop with IEEE
division from restored inputs (sflx_kernel.hip vege_loop / bare_loop).  Every
column must still equal the C restatement of the reference bit for bit, in
both occupancy instantiations and at diagnostics levels NONE and FULL, and
the device counter must show the in-loop windows fired.  A dry-clay set sends
soil-water sub-step divisions (NMP_SOIL_DIV) below DivFast32's exact region:
they must take IEEE division (counted) and stay bit-exact.

    NOAHMP_ENGINE_LIB=.../lib_probe_midloop.so python tests/probe_midloop.py

Prints one JSON line; exit status 0 when every check passed.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from golden_io import bit_equal, load_params  # noqa: E402
from noahmp_amd import cases, layout as L, lib  # noqa: E402
from noahmp_amd.engine import ColumnState, Engine  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402
import port  # noqa: E402  (the oracle: the checker)

# fb_why bits (sflx_kernel.hip NMP_DOM): the windows checked inside the loops
IN_LOOP = {16: "RAHG window", 17: "RSSUN/RSSHA", 19: "TV window (iter >= 2)",
           20: "TGB window (bare)", 26: "CTR numerator", 27: "TR numerator",
           28: "DTV numerator", 29: "DTG numerator (bare)"}


def main():
    raw = lib.load()
    if not hasattr(raw, "nmp_debug_fallback_count"):
        print(json.dumps({"error": f"{lib.library_path()} is not a probe build"}))
        return 2
    raw.nmp_debug_fallback_count.restype = C.c_longlong
    raw.nmp_debug_fallback_count.argtypes = [C.c_int, C.c_void_p]
    P = Params.builtin("STAS", "USGS")
    opts = [L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES]
    n, jul, dt, yl = 8192, 180.3, 1800.0, 366
    res = {"ncol": n, "runs": []}
    ok_all = True
    for seed in (31, 32):
        cols = cases.make_columns(n, "mixed", P.as_dict(), seed=seed, julian=180.0)
        f = cases.forcing_step(cols, jul, yl, 0, seed=seed)
        est, eisn, edg, _ = port.step(load_params(), tuple(opts), cases.CASE_NML_ZSOIL, dt, yl,
                                      jul, cols.state, cols.isnow, cols.static_f, cols.static_i, f)
        for variant in ("small", "full"):
            for level in ("none", "full"):
                eng = Engine(P, L.CASE_NML_OPTIONS, device=0)
                assert eng.launch_variant(variant) == variant
                cs = ColumnState.from_host(cols, "cuda:0")
                raw.nmp_debug_fallback_count(1, None)
                if level == "full":
                    diag = torch.zeros((L.NDIAG_FULL, n), device="cuda:0")
                    eng.step(cs, torch.as_tensor(f, device="cuda:0"), cases.CASE_NML_ZSOIL, dt,
                             jul, yl, diag, L.DIAG_FULL_LEVEL)
                else:
                    eng.step(cs, torch.as_tensor(f, device="cuda:0"), cases.CASE_NML_ZSOIL, dt,
                             jul, yl)
                torch.cuda.synchronize()
                why = np.zeros(32, np.uint32)
                fb = int(raw.nmp_debug_fallback_count(1, why.ctypes.data))
                got = cs.state.cpu().numpy()
                ok = bit_equal(got, est).all(0) & (cs.isnow.cpu().numpy() == eisn)
                if level == "full":
                    ok &= bit_equal(diag.cpu().numpy(), edg).all(0)
                eng.close()
                run = {"seed": seed, "variant": variant, "diag": level, "fallbacks": fb,
                       "in_loop": {IN_LOOP[b]: int(why[b]) for b in IN_LOOP},
                       "columns_differing": int((~ok).sum())}
                res["runs"].append(run)
                ok_all = ok_all and bool(ok.all() and fb > 0 and why[19] > 0 and why[20] > 0
                                         and why[28] > 0 and why[29] > 0)
    # soil water (NMP_SOIL_DIV): very dry clay (SOILTYP 12, BEXP 11.55) makes
    # WDF * DDZ fall below 2^-102, outside DivFast32's exact region: those
    # divisions must take IEEE division (fb_reason[25]) and every column keep
    # the reference's bits
    for seed in (41,):
        cols = cases.make_columns(n, "mixed", P.as_dict(), seed=seed, julian=180.0)
        dry = np.arange(n) % 2 == 0
        si = cols.static_i
        si[L.STATIC_I.index("SOILTYP")][dry] = 12
        for fld in ("SH2O", "SMC"):
            st = cols.state[L.s(fld)]
            st[:, dry] = np.float32(0.001) + np.float32(0.0001) * np.arange(4)[:, None]
        f = cases.forcing_step(cols, jul, yl, 0, seed=seed)
        est, eisn, edg, _ = port.step(load_params(), tuple(opts), cases.CASE_NML_ZSOIL, dt, yl,
                                      jul, cols.state, cols.isnow, cols.static_f, cols.static_i, f)
        for variant in ("small", "full"):
            eng = Engine(P, L.CASE_NML_OPTIONS, device=0)
            assert eng.launch_variant(variant) == variant
            cs = ColumnState.from_host(cols, "cuda:0")
            raw.nmp_debug_fallback_count(1, None)
            diag = torch.zeros((L.NDIAG_FULL, n), device="cuda:0")
            eng.step(cs, torch.as_tensor(f, device="cuda:0"), cases.CASE_NML_ZSOIL, dt, jul, yl,
                     diag, L.DIAG_FULL_LEVEL)
            torch.cuda.synchronize()
            why = np.zeros(32, np.uint32)
            raw.nmp_debug_fallback_count(1, why.ctypes.data)
            ok = bit_equal(cs.state.cpu().numpy(), est).all(0) & \
                (cs.isnow.cpu().numpy() == eisn) & bit_equal(diag.cpu().numpy(), edg).all(0)
            eng.close()
            run = {"seed": seed, "variant": variant, "case": "dry clay",
                   "soil_ieee_divisions": int(why[25]), "columns_differing": int((~ok).sum())}
            res["runs"].append(run)
            ok_all = ok_all and bool(ok.all() and why[25] > 0)
    res["ok"] = ok_all
    print(json.dumps(res))
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
