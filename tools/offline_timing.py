"""The offline driver at scale: the host path north_star
names (the repo's Python driver calling the engine through ctypes), timed on
a 1,048,576-column netCDF case from the namelist's files.

Writes a case (tools/make_offline_case.py: static file, initial state, hourly
LDASIN files without CO2AIR / O2AIR, the standard HRLDAS set) for
examples/offline_case.nml's day (96 steps of 900 s, output every 3 hours),
then runs `OfflineDriver.from_files` over it in each upload mode and
precision: the 12 forcing fields built on the host and uploaded (48 B per
column per step in fp32, 96 in fp64), the LDASIN block (the files' 8
variables + COSZ, fp32, 36 B) expanded on the device (nmp_forcing_from_ldasin),
and that block uploaded once per input file with COSZ formed on the device
(cosz="device", nmp_forcing_from_ldasin_geo: no upload between files), built
on the host or -- the default -- formed on the device from the file's bytes
as stored (ingest, nmp_ldasin_ingest: the host only copies them).
After 4 warm-up steps the remaining steps are timed, wall clock between two
synchronizes, with the driver's own per-phase host times (`phase_s`: LDASIN
file reads, forcing build + upload enqueue, launch enqueue, output gather +
LDASOUT writes).  The engine alone on the same columns with resident forcing
is timed alongside, the ceiling the driver approaches.

    python tools/offline_timing.py --out profiles/r06/offline_driver.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import config, driver, layout as L  # noqa: E402


def write_namelist(d: str) -> str:
    text = open(os.path.join(ROOT, "examples", "offline_case.nml")).read()
    for k in ("geo_em.d01.nc", "init.nc", "ldasin", "ldasout", "restart"):
        text = text.replace(f"'{k}'", f"'{os.path.join(d, k)}'").replace(
            f'"{k}"', f'"{os.path.join(d, k)}"')
    p = os.path.join(d, "case.nml")
    with open(p, "w") as f:
        f.write(text)
    return p


def time_driver(cfg, precision, ldasin, warm, steps, threads, cosz="host", ingest=False):
    import torch
    t0 = time.perf_counter()
    drv = driver.OfflineDriver.from_files(cfg, precision=precision, ldasin_upload=ldasin,
                                          host_threads=threads, cosz=cosz, ingest=ingest)
    setup = time.perf_counter() - t0
    drv.run(nsteps=warm)
    torch.cuda.synchronize()
    drv.phase_s.clear()
    n_written = len(drv.written)
    upl = drv.ingest or drv.raw_upload or drv.upload
    up0 = upl.count
    t0 = time.perf_counter()
    drv.run(nsteps=steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n = drv.cs.ncol
    outs = len(drv.written) - n_written
    puts = upl.count - up0
    bytes_per_put = upl.host[0].numel() * upl.host[0].element_size()
    kind = "12 fields" if drv.raw_upload is None else (
        "file bytes, device ingest + cosz" if drv.ingest is not None else
        "ldasin block + device cosz" if drv.geo is not None else "ldasin block")
    res = {"precision": precision, "upload": kind, "host_threads": threads, "ncol": n,
           "steps": steps, "output_steps": outs, "uploads": puts,
           "wall_s": el, "ms_per_step": el * 1e3 / steps, "colsteps_per_s": n * steps / el,
           "phase_ms_per_step": {k: v * 1e3 / steps for k, v in drv.phase_s.items()},
           "pcie_up_bytes_per_step": bytes_per_put * puts / steps,
           "pcie_down_bytes_per_output_step": L.NDIAG_OUT * precision * n,
           "setup_s": setup,
           "status_nonzero_cols": int((drv.cs.status != 0).sum().item())}
    state = drv.cs.state.cpu().numpy()
    drv.engine.close()
    return res, state, drv


def time_engine(drv_like, precision, steps):
    """The engine alone: the driver's columns (same order), resident forcing
    (one step's fields), two stream ranges, no output."""
    import torch
    from noahmp_amd.engine import StreamShards
    cs, eng = drv_like.cs, driver.Engine(drv_like.engine.params, drv_like.cfg.engine_options(),
                                         0, precision)
    f = drv_like.upload.dev[0] if drv_like.raw_upload is None else drv_like.raw_fbuf[0]
    sh = StreamShards(eng, cs, 2)
    jul = 1.0
    for _ in range(4):
        sh.step(f, drv_like.zsoil, drv_like.dt, jul, 366)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        sh.step(f, drv_like.zsoil, drv_like.dt, jul, 366)
    sh.join()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eng.close()
    return {"precision": precision, "ms_per_step": el * 1e3 / steps,
            "colsteps_per_s": cs.ncol * steps / el}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ny", type=int, default=1024)
    ap.add_argument("--nx", type=int, default=1024)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "nmp_case"))
    ap.add_argument("--warm", type=int, default=4)
    ap.add_argument("--steps", type=int, default=92)
    ap.add_argument("--precisions", default="4,8")
    ap.add_argument("--threads", type=int, default=8, help="host threads of the threaded runs")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    nml = write_namelist(a.dir)
    import make_offline_case
    t0 = time.perf_counter()
    make_offline_case.main([nml, "--ny", str(a.ny), "--nx", str(a.nx), "--kind", "mixed"])
    t_case = time.perf_counter() - t0
    print(f"case written in {t_case:.1f} s", flush=True)
    cfg = config.Config(nml)
    runs, engine = [], []
    for prec in [int(p) for p in a.precisions.split(",")]:
        states = []
        # round 5's path (12 fields, one host thread), the threaded host build,
        # and the LDASIN block expanded on the device
        # and the block once per file with COSZ formed on the device
        for ldasin, threads, cz, ing in ((False, 1, "host", False), (False, a.threads, "host", False),
                                         (True, a.threads, "host", False),
                                         (True, a.threads, "device", False),
                                         (True, a.threads, "device", True)):
            r, st, drv = time_driver(cfg, prec, ldasin, a.warm, a.steps, threads, cz, ing)
            states.append(st)
            r["state_equals_first_run"] = bool(np.array_equal(states[0].view(np.uint8),
                                                              st.view(np.uint8)))
            if cz == "device":  # COSZ from the device's double cosine: columns apart by 1 ulp
                iv = np.uint32 if st.dtype == np.float32 else np.uint64
                r["state_cols_differing_from_first_run"] = int(
                    (states[0].view(iv) != st.view(iv)).any(0).sum())
            print(json.dumps(r), flush=True)
            runs.append(r)
        e = time_engine(drv, prec, a.steps)
        print(json.dumps(e), flush=True)
        engine.append(e)
        del drv
    out = {"case": f"{a.ny} x {a.nx} land points (mixed USGS/STAS columns), examples/"
                   f"offline_case.nml day: 900-s steps, hourly LDASIN, 3-hourly LDASOUT",
           "case_write_s": t_case, "driver": runs, "engine_resident_forcing": engine}
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
