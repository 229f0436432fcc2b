"""Observed operand ranges of every division in the canopy Newton loop.

Runs the C restatement's division-statistics build (oracle/, -DORACLE_DIV_STATS;
the arithmetic is the bit-exact fp32 one) over the benchmark's column sets and
the golden fixtures, and prints per site the smallest and largest |a|, |b|,
|a/b| seen (nonzero, finite) and the share of zero numerators, next to the
limits of DivFast32's exact region (csrc/sflx_math.h): |b| in [2^-126, 2^126],
a = 0 or |a| >= 2^-102, quotient normal.  Evidence beside the per-site proofs
of DESIGN.md ("Division in the canopy loop"), not a proof itself.

    python tools/div_ranges.py [--cols 131072] [--steps 48] [--out profiles/r04/div_ranges.txt]
"""
import argparse
import glob
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import noahmp_pkg  # noqa: E402,F401

SITES = {0: "GRAV/TVIR (sfcdif1)", 1: "TMP1 = kgtv*H/rhocp", 2: "MOL = -FV^3/TMP1",
         3: "MOZ = (ZLVL-ZPD)/MOL", 4: "MOZ2 = (2+Z0H)/MOL", 5: "CM = K^2/CMFM^2",
         6: "CH = K^2/(CMFM*CHFH)", 7: "RAHC: 1/(CH*UR)", 10: "GRAV/TAH (ragrb)",
         11: "TMP1G = k*g/TAH*HG/rhocp", 12: "MOLG = -FV^3/TMP1G", 13: "MOZG = (ZPD-Z0MG)/MOLG",
         14: "CWPC*Z0HG/HCAN", 15: "CWPC*(Z0H+ZPD)/HCAN", 16: "HCAN*EXP(CWPC)/CWPC",
         17: "RAHG = TMPRAH2/KH", 18: "TMPRB = 50CWPC/(1-EXP(-CWPC/2))", 20: "CAH = 1/RAHC",
         21: "CVH = 2VAIE/RB", 22: "CGH = 1/RAHG", 23: "ATA", 24: "BTA", 25: "CAW = 1/RAWC",
         26: "CEW = FWET*VAIE/RB", 27: "LAISUNE/(RB+RSSUN)", 28: "LAISHAE/(RB+RSSHA)",
         29: "CGW = 1/(RAWG+RSURF)", 30: "AEA", 31: "BEA", 32: "CEV", 33: "CTR", 34: "EVC",
         35: "TR", 36: "DTV = B/A", 37: "H", 38: "HG", 39: "QSFC"}


def merge(a, b):
    out = a.copy()
    out[:, [0, 2, 4]] = np.minimum(a[:, [0, 2, 4]], b[:, [0, 2, 4]])
    out[:, [1, 3, 5]] = np.maximum(a[:, [1, 3, 5]], b[:, [1, 3, 5]])
    out[:, 6:] = a[:, 6:] + b[:, 6:]
    return out


def run_set(job):
    import port
    from noahmp_amd import cases, layout as L
    from noahmp_amd.params import Params
    kind, n, nsteps, opt_veg, seed = job
    P = Params.builtin().as_dict()
    port.div_stats(reset=True)
    opts = tuple(dict(L.CASE_NML_OPTIONS, opt_veg=opt_veg)[k] for k in L.OPTION_NAMES)
    cols = cases.make_columns(n, kind, P, seed=seed, julian=180.0)
    st, isn = cols.state, cols.isnow
    for s in range(nsteps):
        jul = (180.0 + s * 1800.0 / 86400.0) % 366
        f = cases.forcing_step(cols, jul, 366, s, seed=seed)
        st, isn, _, _ = port.step(P, opts, cases.CASE_NML_ZSOIL, 1800.0, 366,
                                  float(np.float32(jul)), st, isn, cols.static_f, cols.static_i, f,
                                  precision="4d")
    return port.div_stats()


def run_fixture(path):
    import port
    from golden_io import fixture_params, load
    port.div_stats(reset=True)
    g = load(os.path.basename(path))
    P = fixture_params(g)
    if "forcing" in g and g["forcing"].ndim == 3:
        st, isn = g["state0"], g["isnow0"]
        dt = float(g["dt"])
        for s in range(g["forcing"].shape[0]):
            jul = float(np.float32(float(g["julian0"]) + s * dt / 86400.0))
            st, isn, _, _ = port.step(P, tuple(g["options"]), g["zsoil"], dt, int(g["yearlen"]),
                                      jul, st, isn, g["static_f"], g["static_i"], g["forcing"][s],
                                      precision="4d")
    else:
        port.step(P, tuple(g["options"]), g["zsoil"], float(g["dt"]), int(g["yearlen"]),
                  float(g["julian"]), g["state0"], g["isnow0"], g["static_f"], g["static_i"],
                  g["forcing"], precision="4d")
    return port.div_stats()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cols", type=int, default=131072)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    per = a.cols // a.workers
    jobs = [("mixed", per, a.steps, 1, 1000 + w) for w in range(a.workers)]
    jobs += [("conus", per // 2, a.steps, 1, 2000 + w) for w in range(a.workers)]
    jobs += [("global", per // 2, a.steps, 2, 3000 + w) for w in range(a.workers)]
    fixtures = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "single_*.npz")) +
                      glob.glob(os.path.join(ROOT, "tests", "golden", "traj_*.npz")))
    tot = None
    with ProcessPoolExecutor(a.workers) as ex:
        for r in list(ex.map(run_set, jobs)) + list(ex.map(run_fixture, fixtures)):
            tot = r if tot is None else merge(tot, r)
    lines = [f"division operand ranges, canopy Newton loop (+ bare_flux's sfcdif1 for sites 0-6): "
             f"{a.cols} mixed + {a.cols // 2} conus + {a.cols // 2} global (opt_veg 2) columns x "
             f"{a.steps} steps, and {len(fixtures)} golden fixtures",
             "exact region of DivFast32: |b| in [1.2e-38, 8.5e37], a = 0 or |a| >= 2.0e-31, "
             "|q| in [1.2e-38, 8.5e37]",
             f"{'site':34s} {'min|a|':>9s} {'max|a|':>9s} {'min|b|':>9s} {'max|b|':>9s} "
             f"{'min|q|':>9s} {'max|q|':>9s} {'calls':>10s} {'a=0':>7s}"]
    for k, name in SITES.items():
        r = tot[k]
        if r[6] == 0:
            lines.append(f"{name:34s} (not reached)")
            continue
        lines.append(f"{name:34s} " + " ".join(f"{v:9.2e}" for v in r[:6]) +
                     f" {int(r[6]):10d} {r[7] / r[6]:7.1%}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
