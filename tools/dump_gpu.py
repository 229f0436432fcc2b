"""Run every golden fixture through the GPU engine and save the raw outputs
(gpurun_out/dump/*.npz) for offline comparison with the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from golden_io import load, single_names  # noqa: E402
from noahmp_amd import cases, layout as L  # noqa: E402
from noahmp_amd.engine import ColumnState, Engine  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out", "dump")
os.makedirs(OUT, exist_ok=True)
P = Params.builtin()
DEV = "cuda:0"
engines = {}


def eng(options, prec=4, math="ref"):
    k = (tuple(int(x) for x in options), prec, math)
    if k not in engines:
        engines[k] = Engine(P, dict(zip(L.OPTION_NAMES, k[0])), 0, prec, math)
    return engines[k]


def cs_of(g, dtype):
    cols = cases.ColumnSet(g["static_f"], g["static_i"], g["state0"], g["isnow0"], *([None] * 7))
    return ColumnState.from_host(cols, DEV, dtype)


for name in single_names():
    g = load(f"single_{name}.npz")
    res = {}
    for tag, prec, math in (("ref", 4, "ref"), ("fast", 4, "fast"), ("f64", 8, "ref")):
        dt = torch.float32 if prec == 4 else torch.float64
        cs = cs_of(g, dt)
        d = torch.zeros((L.NDIAG_FULL, cs.ncol), dtype=dt, device=DEV)
        eng(g["options"], prec, math).step(cs, torch.as_tensor(g["forcing"], device=DEV).to(dt),
                                           g["zsoil"], float(g["dt"]), float(g["julian"]),
                                           int(g["yearlen"]), d, L.DIAG_FULL_LEVEL)
        torch.cuda.synchronize()
        res.update({f"{tag}_state": cs.state.cpu().numpy(), f"{tag}_isnow": cs.isnow.cpu().numpy(),
                    f"{tag}_diag": d.cpu().numpy(), f"{tag}_status": cs.status.cpu().numpy()})
    np.savez_compressed(os.path.join(OUT, f"single_{name}.npz"), **res)

for name in ("casenml", "snow"):
    g = load(f"traj_{name}.npz")
    cs = cs_of(g, torch.float32)
    e = eng(g["options"])
    F = torch.as_tensor(g["forcing"], device=DEV)
    d = torch.zeros((L.NDIAG_FULL, cs.ncol), device=DEV)
    S, I, D = [], [], []
    dt = float(g["dt"])
    for s in range(F.shape[0]):
        e.step(cs, F[s], g["zsoil"], dt, float(g["julian0"]) + s * dt / 86400.0, int(g["yearlen"]),
               d, L.DIAG_FULL_LEVEL)
        S.append(cs.state.cpu().numpy())
        I.append(cs.isnow.cpu().numpy())
        D.append(d.cpu().numpy())
    np.savez_compressed(os.path.join(OUT, f"traj_{name}.npz"), states=np.stack(S),
                        isnows=np.stack(I), diags=np.stack(D))
print("dumped to", OUT)
