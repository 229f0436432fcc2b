"""Offline driver end to end on the GPU: namelist -> Config -> time loop ->
engine, over the run/case.nml period (2000-01-01, 96 x 900 s), against the
reference's own run of the same columns and forcing (traj_casenml fixture,
bit for bit), plus output files and a restart round trip."""
import glob
import os

import numpy as np
import pytest
import torch

from golden_io import bit_equal, load
from noahmp_amd import cases, config, driver, layout as L

pytestmark = pytest.mark.gpu


def _cols(g):
    return cases.ColumnSet(g["static_f"], g["static_i"], g["state0"], g["isnow0"], *([None] * 7))


def _cfg(tmp_path):
    from test_config import write_case
    return config.Config(write_case(tmp_path))


def test_driver_reproduces_reference_trajectory(engine_lib, tmp_path):
    g = load("traj_casenml.npz")
    cfg = _cfg(tmp_path)
    fixture_forcing = lambda step, t: g["forcing"][step]  # noqa: E731
    drv = driver.OfflineDriver(cfg, _cols(g), forcing=fixture_forcing)
    drv.run()
    assert drv.step_index == 96 and drv.t == cfg.enddatetime
    st = drv.cs.state.cpu().numpy()
    assert bit_equal(st, g["states"][-1]).all()
    assert np.array_equal(drv.cs.isnow.cpu().numpy(), g["isnows"][-1])
    files = sorted(glob.glob(os.path.join(cfg.outdir, "*.LDASOUT.npz")))
    assert len(files) == 8 and os.path.basename(files[-1]).startswith("2000010200")
    with np.load(files[-1], allow_pickle=False) as z:
        d = z["diag"]
    # the 16 output fluxes of the last step equal the reference's diagnostics
    for i, name in enumerate(L.DIAG_OUT):
        if name != "T2M":
            assert bit_equal(d[i], g["diags"][-1][L.DIAG_FULL.index(name)]).all(), name


def test_restart_round_trip(engine_lib, tmp_path):
    g = load("traj_casenml.npz")
    cfg = _cfg(tmp_path)
    ff = lambda step, t: g["forcing"][step]  # noqa: E731
    a = driver.OfflineDriver(cfg, _cols(g), forcing=ff, write=False).run(nsteps=40)
    path = str(tmp_path / "r.npz")
    a.save_restart(path)
    b = driver.OfflineDriver(cfg, _cols(g), forcing=ff, write=False)
    b.load_restart(path)
    assert b.step_index == 40
    b.run()
    assert bit_equal(b.cs.state.cpu().numpy(), g["states"][-1]).all()
