"""Per-phase wave-cycle split of the sflx kernel (variant lib built with
-DNMP_PHASE_TIMING, see tools/build_variants.py).  Runs the bench workload
for a few steps and prints each phase's share of the accumulated cycles."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NOAHMP_ENGINE_LIB",
                      os.path.join(ROOT, "noahmp-1_amd", "lib", "variants", "lib_phase.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L  # noqa: E402
from noahmp_amd.engine import ColumnState, Engine  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402

NAMES = ["prelude(atm,phenology,fveg,fsno)", "df_top (first-layer conductivity)", "radiation", "btran+rsurf",
         "vege_flux", "bare_flux", "aggregate", "tsnosoi", "phasechange", "canwater",
         "snowwater", "frozen ground", "soilh2o+groundwater", "carbon+checks", "thermoprop", "-"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    kind = sys.argv[2] if len(sys.argv) > 2 else "mixed"
    math = sys.argv[3] if len(sys.argv) > 3 else "ref"
    P = Params.builtin()
    cols = cases.make_columns(n, kind, P.as_dict(), seed=1000, julian=180.0)
    order = sys.argv[4] if len(sys.argv) > 4 else "lon-snow-type"
    if order != "as-generated":  # the bench's default column order
        from noahmp_amd.order import coherent_order
        cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, order))
    precision = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    opt_veg = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    dtype = torch.float32 if precision == 4 else torch.float64
    eng = Engine(P, dict(L.CASE_NML_OPTIONS, opt_veg=opt_veg), 0, precision,
                 math if precision == 4 else "ref")
    lib = eng._lib
    lib.nmp_debug_phase_cycles.argtypes = [C.c_void_p, C.c_int]
    cs = ColumnState.from_host(cols, "cuda:0", dtype)
    F = [torch.as_tensor(cases.forcing_step(cols, 180.0 + s / 48.0, 366, s, seed=1000),
                         device="cuda:0").to(dtype) for s in range(8)]
    buf = (C.c_ulonglong * 16)()
    for s in range(10):
        if s == 2:
            torch.cuda.synchronize()
            lib.nmp_debug_phase_cycles(buf, 1)
        eng.step(cs, F[s % 8], cases.CASE_NML_ZSOIL, 1800.0, 180.0 + s / 48.0, 366)
    torch.cuda.synchronize()
    lib.nmp_debug_phase_cycles(buf, 0)
    v = np.array(list(buf), dtype=np.float64)
    tot = v.sum()
    print(f"ncol={n} kind={kind} math={math} order={order} precision={precision} "
          f"opt_veg={opt_veg}: wave-cycles per column-step "
          f"{tot / (8 * n / 64) / 64:.0f} (per lane-equivalent)")
    for i in np.argsort(-v):
        if v[i] > 0:
            print(f"  {NAMES[i]:36s} {100 * v[i] / tot:5.1f} %")


if __name__ == "__main__":
    main()
