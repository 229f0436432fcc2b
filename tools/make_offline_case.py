"""Write an offline case in the netCDF-3 layouts of noahmp_amd/ncio.py: the
static file, initial state and LDASIN forcing the namelist names, from the
seeded synthetic generator on a regular lat-lon grid.  noahmp_offline.py then
runs it from the files.

    python tools/make_offline_case.py case.nml [--ny 32 --nx 64 --kind conus]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, config, ncio, timeman  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("nmlfile")
    ap.add_argument("--ny", type=int, default=32)
    ap.add_argument("--nx", type=int, default=64)
    ap.add_argument("--lat0", type=float, default=30.0)
    ap.add_argument("--lon0", type=float, default=-120.0)
    ap.add_argument("--dlat", type=float, default=0.25)
    ap.add_argument("--kind", default="conus", choices=("mixed", "conus", "casenml"))
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    cfg = config.Config(a.nmlfile)
    lat = a.lat0 + a.dlat * np.arange(a.ny)[:, None] + 0.0 * np.arange(a.nx)[None, :]
    lon = a.lon0 + a.dlat * np.arange(a.nx)[None, :] + 0.0 * np.arange(a.ny)[:, None]
    grid = ncio.Grid(lat, lon, np.ones((a.ny, a.nx), bool))
    P = Params.builtin().as_dict()
    cols = cases.make_columns(grid.n, a.kind, P, seed=a.seed,
                              julian=timeman.julian(cfg.begdatetime))
    cols.static_f[0] = grid.lat_rad.astype(np.float32)  # LAT from the grid
    cols.lon = grid.lon_rad
    for path in (cfg.constfile, cfg.initfile):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
    os.makedirs(cfg.indir, exist_ok=True)
    ncio.write_static(cfg.constfile, cols, grid)
    ncio.write_state(cfg.initfile, grid, cols.state, cols.isnow, cfg.begdatetime)
    every, t, k = cfg.input_interval, cfg.begdatetime, 0
    while t < cfg.enddatetime:
        f = cases.forcing_step(cols, timeman.julian(t), timeman.yearlen(t.year), k, seed=a.seed)
        ncio.write_ldasin(ncio.ldasin_path(cfg.indir, t), grid, f, t, extras=False)
        t, k = t + every, k + 1
    print(f"{grid.n} columns, {k} LDASIN files in {cfg.indir}; static {cfg.constfile}, "
          f"init {cfg.initfile}")


if __name__ == "__main__":
    main()
