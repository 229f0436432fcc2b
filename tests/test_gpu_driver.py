"""Offline driver end to end on the GPU: namelist -> Config -> time loop ->
engine, over the run/case.nml period (2000-01-01, 96 x 900 s), against the
reference's own run of the same columns and forcing (traj_casenml fixture,
bit for bit), plus output files and a restart round trip."""
import glob
import os

import numpy as np
import pytest
import torch

import noahmp_pkg  # noqa: F401  (spawned ranks re-import this module)
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


def test_driver_from_netcdf_files(engine_lib, tmp_path):
    """namelist -> static / init / LDASIN netCDF files (ncio.py) -> time loop ->
    LDASOUT netCDF and a netCDF restart: the reference trajectory bit for bit.
    The files carry the trajectory's own CO2AIR / O2AIR, so the driver uploads
    the 12-field host form."""
    from noahmp_amd import ncio
    from test_config import write_case
    from test_ncio import grid_for
    g = load("traj_casenml.npz")
    cols = _cols(g)
    grid = grid_for(cols)
    static, init, indir = tmp_path / "geo_em.d01.nc", tmp_path / "init.nc", tmp_path / "ldasin"
    indir.mkdir()
    nml = write_case(tmp_path)
    text = open(nml).read().replace("'geo_em.d01.nc'", f"'{static}'").replace(
        '"init.nc"', f'"{init}"').replace("'ldasin'", f"'{indir}'").replace(
        "'1 hour'", "'900 second'")
    open(nml, "w").write(text)
    cfg = config.Config(nml)
    ncio.write_static(str(static), cols, grid)
    ncio.write_state(str(init), grid, g["state0"], g["isnow0"], cfg.begdatetime)
    for k, t in enumerate([cfg.begdatetime + i * cfg.timestep for i in range(96)]):
        ncio.write_ldasin(ncio.ldasin_path(str(indir), t), grid, g["forcing"][k], t)
    drv = driver.OfflineDriver.from_files(cfg)
    assert np.array_equal(np.sort(drv.perm), np.arange(32))  # the coherent column order
    drv.run()
    assert drv.step_index == 96 and drv.upload.count == 96
    assert bit_equal(drv.to_grid_order(drv.cs.state.cpu().numpy()), g["states"][-1]).all()
    files = sorted(glob.glob(os.path.join(cfg.outdir, "*.LDASOUT_DOMAIN1")))
    assert len(files) == 8
    d = ncio.read_ldasout(files[-1], grid)
    for i, name in enumerate(L.DIAG_OUT):
        if name != "T2M":
            assert bit_equal(d[i], g["diags"][-1][L.DIAG_FULL.index(name)]).all(), name
    # netCDF restart half way, resumed by a fresh driver
    a = driver.OfflineDriver.from_files(cfg, write=False).run(nsteps=40)
    path = str(tmp_path / "RESTART.nc")
    a.save_restart(path)
    b = driver.OfflineDriver.from_files(cfg, init=path, write=False)
    assert b.step_index == 40
    b.run()
    assert bit_equal(b.to_grid_order(b.cs.state.cpu().numpy()), g["states"][-1]).all()
    # grid order (order=None) gives the same bits
    c = driver.OfflineDriver.from_files(cfg, init=path, write=False, order=None).run()
    assert bit_equal(c.cs.state.cpu().numpy(), g["states"][-1]).all()


@pytest.mark.parametrize("precision", [4, 8])
def test_driver_ldasin_block_equals_host_fields(engine_lib, tmp_path, precision):
    """Standard HRLDAS files (the 8 LDASIN variables only; COSZ from the grid,
    CO2AIR / O2AIR from PSFC): the driver uploads the LDASIN block with the
    host's COSZ every step and the engine forms the 12 fields on each range's
    stream (nmp_forcing_from_ldasin, cosz="host"), or uploads each file's
    variables once per input interval and forms COSZ on the device as well
    (nmp_forcing_from_ldasin_geo, cosz="device": 24 uploads for 96 steps) --
    the block built on the host, or the file's bytes uploaded as stored and
    the block formed on the device (nmp_ldasin_ingest, ingest=True) -- or
    builds the 12 fields on the host (ldasin_upload=False).  All four runs
    give the same state, ISNOW and LDASOUT files bit for bit, in fp32 and
    fp64, from two host threads or one.  (The device COSZ equals the host's
    on every one of these 3,072 column-steps -- checked first, so a rounding
    difference of the two double cosines would be named as such.)"""
    from noahmp_amd import ncio
    from test_config import write_case
    from test_ncio import grid_for
    g = load("traj_casenml.npz")
    cols = _cols(g)
    grid = grid_for(cols)
    static, init, indir = tmp_path / "geo_em.d01.nc", tmp_path / "init.nc", tmp_path / "ldasin"
    indir.mkdir()
    nml = write_case(tmp_path)
    text = open(nml).read().replace("'geo_em.d01.nc'", f"'{static}'").replace(
        '"init.nc"', f'"{init}"').replace("'ldasin'", f"'{indir}'")
    open(nml, "w").write(text)
    cfg = config.Config(nml)
    ncio.write_static(str(static), cols, grid)
    ncio.write_state(str(init), grid, g["state0"], g["isnow0"], cfg.begdatetime)
    t = cfg.begdatetime
    for k in range(0, 96, 4):  # hourly files (input_frequency '1 hour')
        ncio.write_ldasin(ncio.ldasin_path(str(indir), t), grid, g["forcing"][k], t, extras=False)
        t = t + cfg.input_interval
    runs = []
    for ldasin, threads, cz, ing in ((False, 1, "host", False), (True, 2, "host", False),
                                     (True, 2, "device", False), (True, 2, "device", True)):
        cfg.outdir = str(tmp_path / f"out_{int(ldasin)}_{cz}_{int(ing)}")
        drv = driver.OfflineDriver.from_files(cfg, precision=precision, ldasin_upload=ldasin,
                                              host_threads=threads, cosz=cz, ingest=ing)
        if cz == "device" and not ing:
            _check_device_cosz_equals_host(drv, cfg, 96)
        drv.run()
        assert drv.step_index == 96
        uploads = 0 if not ldasin else (96 if cz == "host" else 24)
        assert (drv.raw_upload.count if drv.raw_upload is not None else 0) == \
            (0 if ing else uploads)
        assert (drv.ingest.count if drv.ingest is not None else 0) == (uploads if ing else 0)
        assert drv.upload.count == (0 if ldasin else 96)
        outs = [ncio.read_ldasout(f, grid) for f in sorted(
            glob.glob(os.path.join(cfg.outdir, "*.LDASOUT_DOMAIN1")))]
        assert len(outs) == 8
        runs.append((drv.cs.state.cpu().numpy(), drv.cs.isnow.cpu().numpy(), outs))
        drv.engine.close()
    s0, i0, o0 = runs[0]
    for s1, i1, o1 in runs[1:]:
        assert bit_equal(s1, s0).all() and np.array_equal(i1, i0)
        for a, b in zip(o1, o0):
            assert bit_equal(a, b).all()
    assert np.isfinite(s0[L.s("STC")]).all()


def _check_device_cosz_equals_host(drv, cfg, nsteps):
    """The COSZ nmp_forcing_from_ldasin_geo forms for each of the run's steps
    equals the host reader's (timeman.cosz rounded to fp32) on every column."""
    from noahmp_amd import timeman
    fr = drv.forcing
    geo = torch.as_tensor(fr.geo(), device=drv.dev)
    blk = torch.zeros((L.NLDASIN, drv.cs.ncol), dtype=torch.float32, device=drv.dev)
    out = torch.empty((L.NFORCING, drv.cs.ncol), dtype=drv.dtype, device=drv.dev)
    t = cfg.begdatetime
    for k in range(nsteps):
        jul, yl = timeman.julian(t), timeman.yearlen(t.year)
        drv.engine.forcing_from_ldasin(blk, out, geo=geo, solar=timeman.solar_terms(jul, yl))
        got = out[L.FORCING.index("COSZ")].cpu().numpy().astype(np.float32)
        want = timeman.cosz(fr.lat, fr.lon, jul, yl).astype(np.float32)
        assert bit_equal(got, want).all(), f"step {k}: device COSZ differs from the host's"
        t = t + cfg.timestep


def test_offline_cli_runs_a_netcdf_case(engine_lib, tmp_path):
    """tools/make_offline_case.py writes static/init/LDASIN files for the
    namelist; noahmp_offline.py (the run/main.py counterpart) runs them."""
    import importlib.util
    import sys
    from noahmp_amd import ncio
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    nml = tmp_path / "case.nml"
    text = open(os.path.join(root, "examples", "offline_case.nml")).read()
    for k in ("geo_em.d01.nc", "init.nc", "ldasin", "ldasout", "restart"):
        text = text.replace(f"'{k}'", f"'{tmp_path / k}'").replace(f'"{k}"', f'"{tmp_path / k}"')
    nml.write_text(text)
    sys.path.insert(0, os.path.join(root, "tools"))
    import make_offline_case
    make_offline_case.main([str(nml), "--ny", "4", "--nx", "8"])
    spec = importlib.util.spec_from_file_location("noahmp_offline",
                                                  os.path.join(root, "noahmp_offline.py"))
    cli = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cli)
    assert cli.main([str(nml)]) == 0
    files = sorted(glob.glob(str(tmp_path / "ldasout" / "*.LDASOUT_DOMAIN1")))
    assert len(files) == 8
    cfg = config.Config(str(nml))
    from noahmp_amd.params import Params
    grid, _, _ = ncio.read_static(cfg.constfile, Params.builtin().as_dict(), cfg.begdatetime)
    d = ncio.read_ldasout(files[-1], grid)
    assert d.shape == (L.NDIAG_OUT, 32) and np.isfinite(d).all()


def _write_netcdf_case(tmp_path, g, extras=True):
    """static / init / LDASIN files of the traj_casenml columns + a namelist
    (900-s steps); extras=False: standard HRLDAS files (no COSZ / CO2AIR /
    O2AIR), which the driver ingests on the device."""
    from noahmp_amd import ncio
    from test_config import write_case
    from test_ncio import grid_for
    cols = _cols(g)
    grid = grid_for(cols)
    static, init, indir = tmp_path / "geo_em.d01.nc", tmp_path / "init.nc", tmp_path / "ldasin"
    indir.mkdir()
    nml = write_case(tmp_path)
    text = open(nml).read().replace("'geo_em.d01.nc'", f"'{static}'").replace(
        '"init.nc"', f'"{init}"').replace("'ldasin'", f"'{indir}'").replace(
        "'1 hour'", "'900 second'")
    open(nml, "w").write(text)
    cfg = config.Config(nml)
    ncio.write_static(str(static), cols, grid)
    ncio.write_state(str(init), grid, g["state0"], g["isnow0"], cfg.begdatetime)
    for k, t in enumerate([cfg.begdatetime + i * cfg.timestep for i in range(96)]):
        ncio.write_ldasin(ncio.ldasin_path(str(indir), t), grid, g["forcing"][k], t, extras=extras)
    return nml, grid


def _driver_rank(rank, world, port, nml, out_dir):
    """One rank of a multi-rank offline run on the box's single GPU (gloo for
    the gather: RCCL refuses several ranks on one device)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = config.Config(nml)
    drv = driver.OfflineDriver.from_files(cfg)
    drv.run()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), state=drv.cs.state.cpu().numpy(),
             isnow=drv.cs.isnow.cpu().numpy(), cols=drv.cols_index,
             ingest=drv.ingest is not None and drv.ingest.count > 0)
    dist.barrier()
    drv.engine.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_driver_multi_rank_files_equal_reference(engine_lib, tmp_path, world):
    """OfflineDriver.from_files under a process group: each rank reads and
    steps only its shard_range block of the 32 land points in the driver's
    coherent column order (ragged at world 3: 11/11/10), rank 0 gathers
    (shard.DiagGather) and writes LDASOUT for the whole grid in grid order.  Every LDASOUT file and every rank's final state equal the
    reference trajectory bit for bit."""
    import socket
    import torch.multiprocessing as mp
    from noahmp_amd import ncio, shard
    g = load("traj_casenml.npz")
    nml, grid = _write_netcdf_case(tmp_path, g)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_driver_rank, args=(world, port, str(nml), str(tmp_path)), nprocs=world,
                       start_method="spawn")
    cfg = config.Config(str(nml))
    files = sorted(glob.glob(os.path.join(cfg.outdir, "*.LDASOUT_DOMAIN1")))
    assert len(files) == 8
    for j, fn in enumerate(files):
        d = ncio.read_ldasout(fn, grid)
        k = (j + 1) * 12 - 1  # output every 3 hours = 12 steps of 900 s
        for i, name in enumerate(L.DIAG_OUT):
            if name != "T2M":
                assert bit_equal(d[i], g["diags"][k][L.DIAG_FULL.index(name)]).all(), (fn, name)
    seen = []
    for r in range(world):
        s0, cnt = shard.shard_range(32, r, world)
        with np.load(tmp_path / f"rank{r}.npz") as z:
            idx = z["cols"]  # this rank's land points, in the driver's coherent order
            assert z["state"].shape[1] == cnt == idx.size
            assert bit_equal(z["state"], g["states"][-1][:, idx]).all(), r
            assert np.array_equal(z["isnow"], g["isnows"][-1][idx])
            seen.append(idx)
    assert np.array_equal(np.sort(np.concatenate(seen)), np.arange(32))


@pytest.mark.parametrize("world", [2, 3])
def test_driver_multi_rank_ingest_equals_single_rank(engine_lib, tmp_path, world):
    """Standard HRLDAS files under a process group: every rank uploads each
    file's bytes and ingests its own shard on the device (nmp_ldasin_ingest,
    its block of the coherent order), forms COSZ there, and rank 0 gathers
    and writes LDASOUT from the device-formed grids (nmp_ldasout_grid).  The
    LDASOUT files are byte-identical to a single-rank run that builds the 12
    forcing fields on the host, and every rank's final state equals that
    run's columns bit for bit."""
    import socket
    import torch.multiprocessing as mp
    g = load("traj_casenml.npz")
    nml, grid = _write_netcdf_case(tmp_path, g, extras=False)
    cfg = config.Config(str(nml))
    out_multi = cfg.outdir
    cfg.outdir = str(tmp_path / "single")
    one = driver.OfflineDriver.from_files(cfg, ldasin_upload=False).run()
    assert one.upload.count == 96
    ref_state = one.to_grid_order(one.cs.state.cpu().numpy())
    one.engine.close()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_driver_rank, args=(world, port, str(nml), str(tmp_path)), nprocs=world,
                       start_method="spawn")
    multi = sorted(glob.glob(os.path.join(out_multi, "*.LDASOUT_DOMAIN1")))
    single = sorted(glob.glob(os.path.join(cfg.outdir, "*.LDASOUT_DOMAIN1")))
    assert len(multi) == len(single) == 8
    for a, b in zip(multi, single):
        assert os.path.basename(a) == os.path.basename(b)
        assert open(a, "rb").read() == open(b, "rb").read(), a
    for r in range(world):
        with np.load(tmp_path / f"rank{r}.npz") as z:
            assert z["ingest"], "the rank took the device-ingest path"
            assert bit_equal(z["state"], ref_state[:, z["cols"]]).all(), r


def test_driver_device_forcing_equals_engine_steps(engine_lib, tmp_path):
    """OfflineDriver(forcing="device"): each step's forcing generated on the
    device per range (nmp_forcing_synth on the range streams) gives the same
    bits as generating the whole step's forcing in one launch and stepping the
    engine directly."""
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.params import Params
    cfg = _cfg(tmp_path)
    cols = cases.make_columns(50_001, "mixed", Params.builtin().as_dict(), seed=12,
                              julian=timeman_julian(cfg))
    drv = driver.OfflineDriver(cfg, cols, forcing="device", write=False).run(nsteps=10)
    eng = Engine(Params.builtin(), cfg.engine_options(), device=0)
    cs = ColumnState.from_host(cols, "cuda:0")
    clim = torch.as_tensor(cases.climate(cols, np.float32), device="cuda:0")
    f = torch.empty((L.NFORCING, cols.n), device="cuda:0")
    from noahmp_amd import timeman
    t = cfg.begdatetime
    for k in range(10):
        eng.forcing_synth(clim, timeman.julian(t), timeman.yearlen(t.year), 0, k, f)
        eng.step(cs, f, cases.CASE_NML_ZSOIL, cfg.timestep.total_seconds(), timeman.julian(t),
                 timeman.yearlen(t.year))
        t = t + cfg.timestep
    torch.cuda.synchronize()
    assert torch.equal(drv.cs.state.view(torch.int32), cs.state.view(torch.int32))
    assert torch.equal(drv.cs.isnow, cs.isnow)
    eng.close()


def timeman_julian(cfg):
    from noahmp_amd import timeman
    return timeman.julian(cfg.begdatetime)


def _device_forcing_rank(rank, world, port, nml, out_dir, n):
    """One rank of a device-forcing run: its shard_range block of the n columns."""
    import torch.distributed as dist
    from noahmp_amd import shard
    from noahmp_amd.params import Params
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = config.Config(nml)
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=12,
                              julian=timeman_julian(cfg))
    s0, cnt = shard.shard_range(n, rank, world)
    drv = driver.OfflineDriver(cfg, cols.take(np.arange(s0, s0 + cnt)), forcing="device",
                               write=False).run(nsteps=6)
    np.savez(os.path.join(out_dir, f"dev{rank}.npz"), state=drv.cs.state.cpu().numpy())
    dist.barrier()
    drv.engine.close()
    dist.destroy_process_group()


def test_driver_device_forcing_independent_of_world_size(engine_lib, tmp_path):
    """forcing="device" under a process group keys every draw by the global
    column index (first_col = the rank's shard_range start): two ranks give
    each column the forcing, hence the state, of the one-rank run, bit for bit
    (every rank used to draw rank 0's numbers)."""
    import socket
    import torch.multiprocessing as mp
    from noahmp_amd.params import Params
    from test_config import write_case
    n = 20_001
    nml = write_case(tmp_path)
    cfg = config.Config(nml)
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=12,
                              julian=timeman_julian(cfg))
    one = driver.OfflineDriver(cfg, cols, forcing="device", write=False).run(nsteps=6)
    ref = one.cs.state.cpu().numpy()
    one.engine.close()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_device_forcing_rank, args=(2, port, str(nml), str(tmp_path), n),
                       nprocs=2, start_method="spawn")
    got = np.concatenate([np.load(tmp_path / f"dev{r}.npz")["state"] for r in range(2)], axis=1)
    assert bit_equal(got, ref).all()


def test_rccl_gather_path_on_one_gpu(engine_lib):
    """the RCCL branch of the diagnostics gather
    (DiagGather._issue -> all_gather_into_tensor / gather to a root, and
    gather_diag's nccl branches) executed on a world-1 "nccl" group with
    force_collective, inside the bench's double-buffered output loop on a
    comm side stream: every assembled output step equals the plain run's
    diagnostics bit for bit (tests/probe_rccl_gather.py, in a child process
    because it creates a process group)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "probe_rccl_gather.py")],
                       capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, f"probe produced no result (rc {r.returncode}): {r.stderr[-3000:]}"
    res = json.loads(line[-1])
    print(res)
    assert r.returncode == 0 and res["ok"], res


def test_driver_ingest_restart_jump_back(engine_lib, tmp_path):
    """The device-ingest path across a restart loaded into the same driver:
    run 60 steps of standard HRLDAS files (hourly, 4 steps per file: blocks
    resident, the next file read ahead and uploaded beside the steps), load
    the restart written at step 24 and run to the end again.  The final state
    equals an uninterrupted run bit for bit: no block or read-ahead of the
    later time survives the jump into a slot the earlier files reuse."""
    from noahmp_amd import ncio
    from test_config import write_case
    from test_ncio import grid_for
    g = load("traj_casenml.npz")
    cols = _cols(g)
    grid = grid_for(cols)
    static, init, indir = tmp_path / "geo_em.d01.nc", tmp_path / "init.nc", tmp_path / "ldasin"
    indir.mkdir()
    nml = write_case(tmp_path)
    text = open(nml).read().replace("'geo_em.d01.nc'", f"'{static}'").replace(
        '"init.nc"', f'"{init}"').replace("'ldasin'", f"'{indir}'")
    open(nml, "w").write(text)
    cfg = config.Config(nml)
    ncio.write_static(str(static), cols, grid)
    ncio.write_state(str(init), grid, g["state0"], g["isnow0"], cfg.begdatetime)
    t = cfg.begdatetime
    for k in range(0, 96, 4):
        ncio.write_ldasin(ncio.ldasin_path(str(indir), t), grid, g["forcing"][k], t, extras=False)
        t = t + cfg.input_interval
    ref = driver.OfflineDriver.from_files(cfg, write=False).run()
    assert ref.ingest is not None and ref.ingest.count == 24
    want = ref.cs.state.cpu().numpy()
    ref.engine.close()
    drv = driver.OfflineDriver.from_files(cfg, write=False)
    drv.run(nsteps=24)
    path = str(tmp_path / "mid.nc")
    drv.save_restart(path)
    drv.run(nsteps=36)                     # on to step 60, files read ahead
    drv.load_restart(path)                 # back to step 24
    assert drv.step_index == 24 and not drv._blocks
    drv.run()
    assert drv.step_index == 96
    assert bit_equal(drv.cs.state.cpu().numpy(), want).all()
    drv.engine.close()
