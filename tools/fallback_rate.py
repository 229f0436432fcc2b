"""How often a lane leaves the canopy-loop range proof's domain (GPU box).

Loads the `fbcount` build (tools/build_variants.py: the default kernel plus a
device counter of lanes that re-ran the canopy Newton loop with IEEE division)
through NOAHMP_ENGINE_LIB and steps the benchmark's column sets for the
driver's window, printing re-runs per column-step.

    NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_fbcount.so python tools/fallback_rate.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import noahmp_pkg  # noqa: E402,F401


def main():
    import ctypes as C
    import torch
    from noahmp_amd import cases, layout as L, lib
    from noahmp_amd.engine import ColumnState, Engine, StreamShards
    from noahmp_amd.order import coherent_order
    from noahmp_amd.params import Params
    P = Params.builtin("STAS", "USGS")
    raw = lib.load()
    raw.nmp_debug_fallback_count.restype = C.c_longlong
    raw.nmp_debug_fallback_count.argtypes = [C.c_int, C.c_void_p]
    why_names = {0: "SFCTMP/TG", 1: "QAIR/RHOAIR", 2: "SFCPRS/EAIR", 3: "UR", 4: "TMPCM..",
                 5: "ZLVL-ZPD", 6: "HCAN/Z0M/Z0MG/ZPD", 7: "height order", 8: "CWP*VAIE*HCAN",
                 9: "VAIE", 10: "LAISUNE/LAISHAE", 11: "FWET", 12: "FVEG", 13: "SQRT(DLEAF/UC)",
                 14: "RSURF", 16: "RAHG window", 17: "RSSUN/RSSHA", 18: "TV at entry",
                 19: "TV window", 20: "TGB window (bare)", 21: "bare: air/pressure/wind",
                 22: "bare: TMPCM..", 23: "bare: heights/RSURF", 24: "stomata on IEEE",
                 25: "soil-water division on IEEE", 15: "EMG", 26: "CTR numerator",
                 27: "TR numerator", 28: "DTV numerator", 29: "bare: DTG numerator",
                 30: "bare: EMG/CGH"}
    for kind, n, opt_veg, nsteps in (("mixed", 1 << 20, 1, 25), ("conus", 1 << 20, 1, 25),
                                     ("global", 1_036_800, 2, 25), ("casenml", 65536, 1, 96)):
        eng = Engine(P, dict(L.CASE_NML_OPTIONS, opt_veg=opt_veg), device=0)
        cols = cases.make_columns(n, kind, P.as_dict(), seed=1000, julian=180.0)
        if kind != "casenml":
            cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, "lon-snow-type"))
        cs = ColumnState.from_host(cols, "cuda:0")
        sh = StreamShards(eng, cs, 2)
        raw.nmp_debug_fallback_count(1, None)
        for k in range(nsteps):
            jul = (180.0 + k * 1800.0 / 86400.0) % 366
            f = torch.as_tensor(cases.forcing_step(cols, jul, 366, k, seed=1000), device="cuda:0")
            sh.step(f, cases.CASE_NML_ZSOIL, 1800.0, jul, 366)
        sh.join()
        torch.cuda.synchronize()
        why = np.zeros(32, np.uint32)
        fb = raw.nmp_debug_fallback_count(1, why.ctypes.data)
        print(f"{kind:8s} {n:8d} columns x {nsteps} steps: {fb} IEEE loop re-runs (canopy + bare) "
              f"({fb / (n * nsteps):.2e} per column-step), status bits "
              f"{int((cs.status != 0).sum())}", flush=True)
        print("   by condition:", {why_names.get(b, b): int(why[b]) for b in range(32) if why[b]},
              flush=True)
        eng.close()


if __name__ == "__main__":
    main()
