"""Ceiling probe (not a product path): does laying config #3 out by the
canopy loop's trip counts, on top of the coherent order, shorten the step?

Builds the bench's config #3 column set in its coherent order
(lon-snow-type, 4-degree bands), runs `--warm` steps recording each column's
vege_flux trip count (nmp_step_binned's `cost` with the identity order), then
times `--steps` steps three ways, each from the same post-warm-up state:
  coherent      the layout the bench uses
  trips         columns re-laid once by (band, snow, type, trip-count bucket)
                of the last warm-up step (a physical permutation of state,
                static fields and the resident forcing)
  trips_global  re-laid by the trip count alone (ignoring the coherent key)
Prints ms per step (HIP events around the timed steps) for each.

--from-start: the layout decided at set-up instead, from the trip counts of
ONE probe step on a scratch copy of the initial state (as a run's driver
could do before its first step), then `--warm` + `--steps` steps on it from
the initial state, against the coherent layout under the same protocol.

    python tools/trip_order_probe.py [--warm 5] [--steps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L  # noqa: E402
from noahmp_amd.engine import ColumnState, Engine, StreamShards  # noqa: E402
from noahmp_amd.order import coherent_order  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncol", type=int, default=1 << 20)
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--period", type=int, default=48)
    ap.add_argument("--from-start", action="store_true")
    a = ap.parse_args()
    if a.from_start:
        return from_start(a)
    dev = "cuda:0"
    P = Params.builtin("STAS", "USGS")
    n, dt, jul0, yl, seed = a.ncol, 1800.0, 180.0, 366, 1000
    cols = cases.make_columns(n, "mixed", P.as_dict(), seed=seed, julian=jul0)
    cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, "lon-snow-type",
                                    band_deg=4.0))
    F = torch.stack([torch.from_numpy(cases.forcing_step(
        cols, (jul0 + s * dt / 86400.0) % yl, yl, s, seed=seed)) for s in range(a.period)]).float().to(dev)
    eng = Engine(P, L.CASE_NML_OPTIONS, device=0, precision=4)
    cs = ColumnState.from_host(cols, dev, torch.float32)
    order = torch.arange(n, dtype=torch.int32, device=dev)
    cost = torch.zeros(n, dtype=torch.uint8, device=dev)
    zs = cases.CASE_NML_ZSOIL
    for k in range(a.warm):
        eng.step(cs, F[k % a.period], zs, dt, jul0 + k * dt / 86400.0, yl, order=order, cost=cost)
    torch.cuda.synchronize()
    trips = cost.cpu().numpy().astype(np.int64)
    band = np.floor(np.degrees(cols.lon) / 4.0).astype(np.int64)
    snow = (cs.isnow.cpu().numpy() < 0)
    vt = cols.static_i[L.STATIC_I.index("VEGTYP")]
    perms = {"coherent": np.arange(n),
             "trips": np.lexsort((trips // 4, vt, snow, band)),
             "trips_global": np.argsort(-trips, kind="stable")}
    base = {f: getattr(cs, f).clone() for f in ("state", "isnow", "static_f", "static_i",
                                                 "status")}
    out = {}
    for name, p in perms.items():
        pt = torch.as_tensor(p, device=dev)
        c2 = ColumnState.from_host(cols, dev, torch.float32)
        for f, t in base.items():
            getattr(c2, f).copy_(t.index_select(t.dim() - 1, pt))
        F2 = F.index_select(2, pt)
        sh = StreamShards(eng, c2, 2)
        diag = torch.zeros((L.NDIAG_OUT, n), device=dev)
        sh.step(F2[a.warm % a.period], zs, dt, jul0 + a.warm * dt / 86400.0, yl)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(a.warm + 1, a.warm + 1 + a.steps):
            out_step = (k + 1) % 6 == 0
            sh.step(F2[k % a.period], zs, dt, jul0 + k * dt / 86400.0, yl,
                    diag if out_step else None, L.DIAG_OUT_LEVEL if out_step else L.DIAG_NONE)
        sh.join()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / a.steps
        # the wave maximum of the recorded trip counts, per 64-column wave, in this layout
        tw = trips[p][: n // 64 * 64].reshape(-1, 64)
        print(json.dumps({"layout": name, "ms_per_step": out[name],
                          "warmup_trips_wave_max_mean": float(tw.max(1).mean()),
                          "warmup_trips_lane_mean": float(tw.mean())}), flush=True)
        del c2, F2, sh
    eng.close()
    return 0


def from_start(a):
    dev = "cuda:0"
    P = Params.builtin("STAS", "USGS")
    n, dt, jul0, yl, seed = a.ncol, 1800.0, 180.0, 366, 1000
    cols = cases.make_columns(n, "mixed", P.as_dict(), seed=seed, julian=jul0)
    cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, "lon-snow-type",
                                    band_deg=4.0))
    F = torch.stack([torch.from_numpy(cases.forcing_step(
        cols, (jul0 + s * dt / 86400.0) % yl, yl, s, seed=seed))
        for s in range(a.period)]).float().to(dev)
    eng = Engine(P, L.CASE_NML_OPTIONS, device=0, precision=4)
    zs = cases.CASE_NML_ZSOIL
    scratch = ColumnState.from_host(cols, dev, torch.float32)
    order = torch.arange(n, dtype=torch.int32, device=dev)
    cost = torch.zeros(n, dtype=torch.uint8, device=dev)
    eng.step(scratch, F[0], zs, dt, jul0, yl, order=order, cost=cost)
    torch.cuda.synchronize()
    trips = cost.cpu().numpy().astype(np.int64)
    del scratch
    band = np.floor(np.degrees(cols.lon) / 4.0).astype(np.int64)
    snow = cols.isnow < 0
    vt = cols.static_i[L.STATIC_I.index("VEGTYP")]
    perms = {"coherent": np.arange(n), "trips_setup": np.lexsort((trips // 4, vt, snow, band)),
             "trips_setup_b2": np.lexsort((trips // 2, vt, snow, band)),
             "trips_setup_b8": np.lexsort((trips // 8, vt, snow, band))}
    for rep in range(2):
        for name, p in perms.items():
            pt = torch.as_tensor(p, device=dev)
            c2 = ColumnState.from_host(cols.take(p), dev, torch.float32)
            F2 = F.index_select(2, pt)
            sh = StreamShards(eng, c2, 2)
            diag = torch.zeros((L.NDIAG_OUT, n), device=dev)

            def step(k):
                out_step = (k + 1) % 6 == 0
                sh.step(F2[k % a.period], zs, dt, jul0 + k * dt / 86400.0, yl,
                        diag if out_step else None,
                        L.DIAG_OUT_LEVEL if out_step else L.DIAG_NONE)
            for k in range(a.warm):
                step(k)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(a.warm, a.warm + a.steps):
                step(k)
            sh.join()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"rep": rep, "layout": name, "from": "set-up probe step",
                              "ms_per_step": e0.elapsed_time(e1) / a.steps}), flush=True)
            del c2, F2, sh
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
