"""Loop trip counts of the bench workload, per lane and per 64-lane wave.

Builds the C oracle with -DORACLE_ITER_STATS (into /tmp), runs `--steps`
steps of the bench's mixed column set and reports, per data-dependent loop,
the mean trip count per column and the mean over waves (64 consecutive
columns) of the slowest lane -- the count the GPU wave actually executes.
mean/max is the lane utilisation of that loop.  CPU only (test-side tool).
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402
import port  # noqa: E402

NAMES = ["vege_flux Newton", "stomata bisection", "frh2o", "soilwater sub-steps",
         "bare_flux Newton"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncol", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--kind", default="mixed")
    ap.add_argument("--order", default=None, help="sort columns by this stats counter index")
    a = ap.parse_args()
    so = "/tmp/liboracle_stats.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-std=c11",
                    "-DORACLE_REAL=float", "-DORACLE_ITER_STATS", "-I", os.path.join(ROOT, "include"),
                    "-shared", "-o", so, os.path.join(ROOT, "oracle", "noahmp_oracle.c"), "-lm"],
                   check=True)
    port.LIBS["cr"] = so  # loaded through port's fp32 binding
    lib, _ = port._lib("cr")
    lib.oracle_set_stats.argtypes = [C.c_void_p]
    P = Params.builtin().as_dict()
    julian0, yearlen, seed, dt = 180.0, 366, 1000, 1800.0
    cols = cases.make_columns(a.ncol, a.kind, P, seed=seed, julian=julian0)
    opts = [L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES]
    st, isn = cols.state.astype(np.float32), cols.isnow.copy()
    tot = np.zeros((a.ncol, 8), np.int64)
    for s in range(a.steps):
        buf = np.zeros((a.ncol, 8), np.int32)
        lib.oracle_set_stats(buf.ctypes.data)
        f = cases.forcing_step(cols, julian0 + s * dt / 86400.0, yearlen, s, seed=seed)
        st, isn, _, _ = port.step(P, opts, cases.CASE_NML_ZSOIL, dt, yearlen,
                                  julian0 + s * dt / 86400.0, st, isn, cols.static_f,
                                  cols.static_i, f, precision="cr")
        tot += buf
        lib.oracle_set_stats(None)
        w = buf[: a.ncol // 64 * 64].reshape(-1, 64, 8)
        day = float(np.mean(f[L.FORCING.index("COSZ")] > 0))
        print(f"step {s} (daylit {day:.2f}):", "  ".join(
            f"{NAMES[k].split()[0]} {w[..., k].mean():.2f}/{w[..., k].max(1).mean():.2f}"
            for k in range(5)))
    w = tot[: a.ncol // 64 * 64].reshape(-1, 64, 8)
    print(f"\n{a.steps} steps, {a.ncol} {a.kind} columns: loop  mean/lane  mean wave-max  util")
    for k in range(5):
        m, mx = w[..., k].mean(), w[..., k].max(1).mean()
        print(f"  {NAMES[k]:22s} {m:8.2f} {mx:8.2f}   {m / mx if mx else 0:.2f}")
    v = tot[:, 0] if a.steps == 1 else None
    h = np.bincount(buf[:, 0], minlength=21)
    print("vege_flux trip histogram (last step):", h.tolist())
    for K in (6, 7, 8, 10, 12):
        frac = float((buf[:, 0] > K).mean())
        wmax = np.minimum(buf[: a.ncol // 64 * 64, 0].reshape(-1, 64), K).max(1).mean()
        print(f"  cap {K:2d}: columns over cap {100 * frac:5.2f} %  capped wave-max {wmax:.2f}")


if __name__ == "__main__":
    main()
