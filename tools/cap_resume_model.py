"""Model of a "cap and resume" split of the canopy Newton loop (VERDICT r4
item 1; CPU only, test-side tool).

The wave runs its slowest lane through vege_flux's Newton loop
(func.f90:2744-2877).  The split: the step kernel stops every lane at
iteration K; a lane still iterating writes its loop context to an HBM side
buffer and leaves the step; a second, compacted launch (64 such columns per
wave) restores the context, runs the remaining iterations and the rest of the
step.  Nothing before the loop and none of the first K iterations is repeated.

Inputs:
  * per-column trip counts of the loop from the C oracle built with
    ORACLE_ITER_STATS (the same counts the kernel runs: the `cost` key equals
    them, test_cost_key_is_the_reference_trip_count), over --steps steps of
    the bench's mixed set in the bench's column order (coherent, 4 degree
    bands, --order as-generated for the generator's order);
  * the step's phase split measured on the GPU (tools/phase_profile.py,
    profiles/r04/phase_mixed.txt): pre-loop 21.5 %, the loop 26.1 %, after the
    loop 52.4 % of wave time;
  * the loop's cost per wave = c1 + c * (m - 1) for a wave-max of m
    iterations, c1 the first iteration (it alone runs the two stomata
    bisections).  c1 / c is not measured: the model is run for c1 = 1, 3 and 6
    times c, and the loop's measured share fixes c.

Costs are wave time in units of the measured step.  Baseline = pre + loop +
post.  Split = pre + loop(min(m, K)) + post for every wave of the main launch
(a wave whose lanes all leave still runs pre and the first K iterations) +
for the resume launch, per compacted wave: restore + c * max(remaining) +
post.  The restore (context reload) and the extra launch are charged as
`--restore` (fraction of the step per resume wave, default 0.02).

    python tools/cap_resume_model.py --ncol 65536 --steps 6
"""
import argparse
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L  # noqa: E402
from noahmp_amd.order import coherent_order  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402
import port  # noqa: E402

PRE, LOOP, POST = 0.215, 0.261, 0.524   # profiles/r04/phase_mixed.txt


def trip_counts(ncol, steps, order):
    so = "/tmp/liboracle_stats.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-std=c11",
                    "-DORACLE_REAL=float", "-DORACLE_ITER_STATS", "-I", os.path.join(ROOT, "include"),
                    "-shared", "-o", so, os.path.join(ROOT, "oracle", "noahmp_oracle.c"), "-lm"],
                   check=True)
    port.LIBS["cr"] = so
    lib, _ = port._lib("cr")
    import ctypes as C
    lib.oracle_set_stats.argtypes = [C.c_void_p]
    P = Params.builtin().as_dict()
    julian0, yearlen, seed, dt = 180.0, 366, 1000, 1800.0
    cols = cases.make_columns(ncol, "mixed", P, seed=seed, julian=julian0)
    if order != "as-generated":
        cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, order, band_deg=4.0))
    opts = [L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES]
    st, isn = cols.state.astype(np.float32), cols.isnow.copy()
    out = []
    for s in range(steps):
        buf = np.zeros((ncol, 8), np.int32)
        lib.oracle_set_stats(buf.ctypes.data)
        jul = julian0 + s * dt / 86400.0
        f = cases.forcing_step(cols, jul, yearlen, s, seed=seed)
        st, isn, _, _ = port.step(P, opts, cases.CASE_NML_ZSOIL, dt, yearlen, jul, st, isn,
                                  cols.static_f, cols.static_i, f, precision="cr")
        lib.oracle_set_stats(None)
        out.append(buf[:, 0].copy())
    return np.stack(out)


def loop_cost(m, c, c1):
    """Wave cost of the loop at wave-max m iterations (0 = no canopy lane)."""
    m = np.asarray(m, np.float64)
    return np.where(m > 0, c1 + c * np.maximum(m - 1, 0), 0.0)


def model(trips, K, ratio, restore):
    """Step time of the split relative to the current kernel (1 = same)."""
    nw = trips.shape[1] // 64
    t = trips[:, :nw * 64]
    wmax = t.reshape(t.shape[0], nw, 64).max(2)
    mean_wmax = wmax.mean()
    # c from the measured loop share: LOOP = mean over waves of c1 + c (m - 1)
    c = LOOP / np.mean(np.where(wmax > 0, ratio + np.maximum(wmax - 1, 0), 0.0))
    c1 = ratio * c
    base = PRE + POST + loop_cost(wmax, c, c1).mean()
    main = PRE + POST + loop_cost(np.minimum(wmax, K), c, c1).mean()
    res_cost, capped = 0.0, 0
    for s in range(t.shape[0]):
        over = t[s][t[s] > K] - K          # remaining iterations, in column order
        capped += over.size
        nr = (over.size + 63) // 64
        if nr == 0:
            continue
        pad = np.zeros(nr * 64, np.int64)
        pad[:over.size] = over
        rem = pad.reshape(nr, 64).max(1)
        res_cost += float(np.sum(restore + c * rem + POST))
    res = res_cost / (t.shape[0] * nw)
    return {"K": K, "c1/c": ratio, "mean_wave_max": mean_wmax, "capped_frac": capped / t.size,
            "main": main / base, "resume": res / base, "total": (main + res) / base}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncol", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--order", default="lon-snow-type")
    ap.add_argument("--restore", type=float, default=0.02)
    a = ap.parse_args()
    trips = trip_counts(a.ncol, a.steps, a.order)
    t = trips[:, :a.ncol // 64 * 64]
    wmax = t.reshape(t.shape[0], -1, 64).max(2)
    print(f"{a.ncol} mixed columns x {a.steps} steps, order {a.order}: trips per lane "
          f"{t.mean():.2f}, wave-max {wmax.mean():.2f}, lane utilisation of the loop "
          f"{t.mean() / wmax.mean():.3f}; share of waves with a 20-iteration lane "
          f"{(wmax == 20).mean():.3f}")
    print(f"phase split (profiles/r04/phase_mixed.txt): pre {PRE}, loop {LOOP}, post {POST}; "
          f"restore per resume wave {a.restore}")
    print(" K   c1/c  capped %  main    resume  total (1 = current kernel)")
    best = None
    for ratio in (1.0, 3.0, 6.0):
        for K in (6, 8, 10, 12, 14, 16):
            r = model(trips, K, ratio, a.restore)
            print(f"{K:2d}  {ratio:4.1f}  {100 * r['capped_frac']:6.2f}  {r['main']:.3f}  "
                  f"{r['resume']:.3f}  {r['total']:.3f}")
            if best is None or r["total"] < best["total"]:
                best = r
    print(f"best: K = {best['K']} at c1/c = {best['c1/c']}: {100 * (1 / best['total'] - 1):+.1f} % "
          "throughput")


if __name__ == "__main__":
    main()
