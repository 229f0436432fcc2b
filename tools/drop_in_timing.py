"""Time the Fortran engine slot (INTEGRATION.md `module noahmp_engine`) at a
production column count (GPU box).

Writes the bench's mixed column set (65,536 columns, case.nml options, 4
forcing steps from julian 180, dt 1800 s) as the drop-in program's input,
then runs `tests/lib/engine_drop_in time` (the module compiled verbatim from
INTEGRATION.md) at --ncol columns (the set replicated) for --steps timed
noahmp_run calls, with the module's arrays page-locked or pageable, and the
16 output fluxes copied back every step or every 6th step (the namelist's
3-hour output at dt = 1800 s), and noahmp_run pipelined over 1-8 column
chunks, with the 12 forcing fields uploaded or the 9-field LDASIN block
(`nmp_ldasin_forcing`, the forcing formed on the device).  Prints one JSON
line per configuration and writes them all to --out.

    python tools/drop_in_timing.py --ncol 1048576 --steps 20 --out gpurun_out/dropin.json
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncol", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--configs", default="1:6:1,1:6:2,1:6:4,1:6:8,1:1:4,0:6:4,1:6:4:1,1:1:4:1,"
                                          "1:6:8:1,1:6:4:2,1:6:2:2,1:6:1:2",
                    help="pinned:out_every:chunks[:ldasin],...; ldasin 2: COSZ only on 3 "
                         "steps of 4")
    a = ap.parse_args()
    exe = os.path.join(ROOT, "tests", "lib", "engine_drop_in")
    tbl = os.path.join(ROOT, "oracle", "_ref", "tbl")
    n, nf, dt, jul0, yl, seed = 65536, 4, 1800.0, 180.0, 366, 1000
    P = Params.builtin()
    cols = cases.make_columns(n, "mixed", P.as_dict(), seed=seed, julian=jul0)
    jul = np.array([jul0 + s * dt / 86400.0 for s in range(nf)], np.float32)
    frc = np.stack([cases.forcing_step(cols, float(jul[s]), yl, s, seed=seed) for s in range(nf)])
    opts = np.array([L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES], np.int32)
    res = []
    with tempfile.TemporaryDirectory() as td:
        fin = os.path.join(td, "in.bin")
        with open(fin, "wb") as f:
            for x in (np.array([n, nf, yl], np.int32), opts,
                      np.asarray(cases.CASE_NML_ZSOIL, np.float32), np.array([dt], np.float32),
                      jul, cols.static_i.astype(np.int32), cols.isnow.astype(np.int32),
                      cols.static_f.astype(np.float32), cols.state.astype(np.float32),
                      frc.astype(np.float32)):
                f.write(np.ascontiguousarray(x).tobytes())
        for cfg in a.configs.split(","):
            pinned, oe, chunks, ldasin = (tuple(int(v) for v in cfg.split(":")) + (0,))[:4]
            fout = os.path.join(td, "t.txt")
            r = subprocess.run([exe, "time", tbl, fin, fout, str(a.ncol), str(a.steps), str(oe),
                                str(pinned), str(chunks), str(ldasin)], capture_output=True, text=True,
                               timeout=300)
            if r.returncode != 0:
                print(r.stdout + r.stderr, file=sys.stderr)
                return r.returncode
            v = open(fout).read().split()
            d = {"ncol": int(v[0]), "steps": int(v[1]), "out_every": int(v[2]),
                 "pinned": bool(int(v[3])), "ms_per_noahmp_run": float(v[4]),
                 "ms_host_forcing_fill": float(v[5]), "column_steps_per_s": float(v[6]),
                 "pcie_bytes_up_per_step": float(v[7]), "pcie_bytes_down_per_step": float(v[8]),
                 "chunks": int(v[9]),
                 "forcing_upload": {0: "12 fields", 1: "ldasin block",
                                    2: "ldasin block, COSZ only between files"}[int(v[10])]}
            d["pcie_gb_per_s"] = (d["pcie_bytes_up_per_step"] + d["pcie_bytes_down_per_step"]) \
                / (d["ms_per_noahmp_run"] * 1e-3) / 1e9
            print(json.dumps(d), flush=True)
            res.append(d)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
