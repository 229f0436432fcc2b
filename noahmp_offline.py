#!/usr/bin/env python3
"""Offline Noah-MP run on the MI355X engine: counterpart of run/main.py.

    python noahmp_offline.py [case.nml] [--ncol N] [--kind casenml|mixed|conus]
                             [--device D] [--restart FILE]

Reads the namelist like the reference (noahmp_amd.config.Config ==
offline/noahmp_config.Config) and then does what the reference driver does
not yet do: runs the time loop through the engine (noahmp_amd.driver).

When the namelist's static_parameter_file exists, the run comes from files
(netCDF-3, noahmp_amd/ncio.py): grid and surface types from the static file,
the state from initialization_file (or --restart), forcing from the LDASIN
files in input_directory; output goes to LDASOUT files.
`tools/make_offline_case.py` writes such a set from the synthetic generator.
Otherwise the columns and forcing are the seeded synthetic set (`--kind
casenml` = the run/case.nml column of SURVEY 8d config #1, replicated --ncol
times).
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, config, driver, timeman  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402

DEFAULT_NAMELIST_FILE = "case.nml"


def main(argv=None):
    ap = argparse.ArgumentParser(description="Noah-MP Land Surface Model (MI355X engine)")
    ap.add_argument("nmlfile", nargs="?", default=DEFAULT_NAMELIST_FILE, help="configuration file")
    ap.add_argument("--ncol", type=int, default=1)
    ap.add_argument("--kind", default="casenml", choices=("casenml", "mixed", "conus", "global"))
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--restart", default=None, help="restart file to start from")
    ap.add_argument("--device-forcing", action="store_true",
                    help="synthetic cases: generate the forcing on the GPU every step "
                         "(nmp_forcing_synth) instead of on the host")
    ap.add_argument("--precision", type=int, default=4, choices=(4, 8),
                    help="engine precision (fp32, the reference's, or fp64)")
    ap.add_argument("--cosz", default="device", choices=("device", "host"),
                    help="netCDF cases: COSZ formed on the device from the grid (default) or "
                         "computed on the host and uploaded every step")
    ap.add_argument("--no-ingest", action="store_true",
                    help="netCDF cases: build each LDASIN block on the host instead of "
                         "uploading the file's bytes for the device to select and order")
    a = ap.parse_args(argv)
    cfg = config.Config(a.nmlfile)
    P = Params.builtin()
    if os.path.isfile(cfg.constfile):
        drv = driver.OfflineDriver.from_files(cfg, device=a.device, params=P, init=a.restart,
                                              precision=a.precision, cosz=a.cosz,
                                              ingest=not a.no_ingest)
        a.ncol = drv.cs.ncol
    else:
        cols = cases.make_columns(a.ncol, a.kind, P.as_dict(), seed=0,
                                  julian=timeman.julian(cfg.begdatetime))
        drv = driver.OfflineDriver(cfg, cols, device=a.device, params=P,
                                   forcing="device" if a.device_forcing else None,
                                   precision=a.precision)
        if a.restart:
            drv.load_restart(a.restart)
    t0 = time.perf_counter()
    drv.run()
    el = time.perf_counter() - t0
    print(f"{drv.step_index} steps x {a.ncol} columns to {drv.t.isoformat()} in {el:.2f} s; "
          f"{len(drv.written)} output files in {cfg.outdir}; status bits set on "
          f"{int((drv.cs.status != 0).sum())} columns")
    return 0


if __name__ == "__main__":
    sys.exit(main())
