"""The file-format kernels around the step (GPU box): per-launch time and
achieved HBM bandwidth against their algorithmic bytes, at 1,048,576 columns.

  forcing_from_ldasin      reads the 9-row fp32 block (36 B), writes 12 fields
                           (48 B fp32 / 96 B fp64)
  forcing_from_ldasin_geo  reads 8 rows (32 B) + geo (24 B), writes 12 fields;
                           one double cosine per column
  ldasin_ingest            reads 8 gathered 4-byte words + the point (36 B),
                           writes 8 rows (32 B)
  ldasout_grid             fills 16 grids (64 B per grid point), then reads 16
                           fluxes + the point (68 B) and scatters them (64 B)

The two gather/scatter kernels are timed with the grid points in the
columns' own order (`point` = identity: coalesced) and fully shuffled (every
lane a different cache line: the worst case; the driver's coherent order lies
between, mostly runs of neighbouring points).  Times are HIP events around
`--reps` back-to-back launches on one stream (mean per launch); run under
`rocprofv3 --kernel-trace --stats` for the kernels' own durations.  Prints
one JSON line per kernel, precision and point order.

    python tools/io_kernels_bench.py [--ncol 1048576] [--reps 50]
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
from noahmp_amd import layout as L, timeman  # noqa: E402
from noahmp_amd.engine import Engine  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402

PEAK_GBS = 8000.0  # MI355X HBM3E (/opt/skills/guides/MI355X_MICROARCH.md)


def timed(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncol", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    n, dev = a.ncol, "cuda:0"
    rng = np.random.default_rng(0)
    npts = n
    points = {"identity": torch.arange(n, dtype=torch.int32, device=dev),
              "shuffled": torch.as_tensor(rng.permutation(npts)[:n].astype(np.int32), device=dev)}
    lat = np.radians(rng.uniform(-60, 70, n))
    lon = np.radians(rng.uniform(-180, 180, n))
    geo = torch.as_tensor(np.stack([np.sin(lat), np.cos(lat), lon]), device=dev)
    blk = torch.as_tensor(rng.uniform(1, 2, (L.NLDASIN, n)).astype(np.float32), device=dev)
    grid_be = torch.as_tensor(rng.integers(0, 2**31 - 1, (L.NLDASIN - 1, npts), dtype=np.int32),
                              device=dev)
    solar = timeman.solar_terms(172.5, 366)
    out = []
    for prec in (4, 8):
        eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=prec)
        dt = torch.float32 if prec == 4 else torch.float64
        f = torch.empty((L.NFORCING, n), dtype=dt, device=dev)
        diag = torch.as_tensor(rng.normal(size=(L.NDIAG_OUT, n)), device=dev).to(dt)
        grids = torch.empty((L.NDIAG_OUT, npts), device=dev,
                            dtype=torch.int32 if prec == 4 else torch.int64)
        cases = [
            ("forcing_from_ldasin", None, lambda: eng.forcing_from_ldasin(blk, f),
             n * (36 + 12 * prec)),
            ("forcing_from_ldasin_geo", None, lambda: eng.forcing_from_ldasin(blk, f, geo=geo,
                                                                              solar=solar),
             n * (32 + 24 + 12 * prec)),
        ]
        for order, pt in points.items():
            cases.append(("ldasout_grid", order,
                          lambda pt=pt: eng.ldasout_grid(diag, pt, grids, -9999.0),
                          npts * 16 * prec + n * (16 * prec + 4 + 16 * prec)))
            if prec == 4:
                cases.append(("ldasin_ingest", order,
                              lambda pt=pt: eng.ldasin_ingest(grid_be, pt, blk),
                              n * (32 + 4 + 32)))
        for name, order, fn, nbytes in cases:
            ms = timed(fn, a.reps)
            gbs = nbytes / (ms * 1e-3) / 1e9
            r = {"kernel": name, "precision": prec, "ncol": n, "point_order": order,
                 "ms_per_launch": ms, "algorithmic_bytes": nbytes, "achieved_gb_s": gbs,
                 "hbm_frac": gbs / PEAK_GBS}
            print(json.dumps(r), flush=True)
            out.append(r)
        eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
