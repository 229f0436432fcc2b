"""netCDF-3 files of the offline run (noahmp_amd/ncio.py): static grid, state
(initialization / restart), LDASIN forcing, LDASOUT output -- host side only.

The reference names these files in run/case.nml:2-11 but has no reader or
writer; the round trips below pin our own layouts (HRLDAS conventions)."""
import datetime

import numpy as np
import pytest

from golden_io import load
from noahmp_amd import cases, layout as L, ncio, timeman

T0 = datetime.datetime(2000, 1, 1)


def bits(a):
    a = np.asarray(a)
    return a.view(np.int32 if a.dtype == np.float32 else np.int64)


def fixture_grid(n, shape=(5, 8), seed=0):
    """A grid whose land mask has n points; lat/lon of the land points given later."""
    rng = np.random.default_rng(seed)
    mask = np.zeros(shape[0] * shape[1], bool)
    mask[np.sort(rng.choice(mask.size, n, replace=False))] = True
    return mask.reshape(shape)


def grid_for(cols, shape=(5, 8), seed=0):
    mask = fixture_grid(cols.n, shape, seed)
    g0 = ncio.Grid(np.zeros(shape), np.zeros(shape), mask)
    lat = g0.scatter(np.degrees(cols.static_f[L.STATIC_F.index("LAT")].astype(np.float64)), 0.0)
    lon = g0.scatter(np.degrees(np.linspace(-2.0, 2.0, cols.n)), 0.0)
    return ncio.Grid(lat, lon, mask)


def test_static_round_trip(tmp_path, ref_params):
    cols = cases.make_columns(32, "conus", ref_params, seed=4)
    grid = grid_for(cols)
    p = str(tmp_path / "geo_em.d01.nc")
    ncio.write_static(p, cols, grid)
    g2, sf, si = ncio.read_static(p, ref_params, T0)
    assert g2.n == 32 and np.array_equal(g2.index, grid.index)
    assert np.array_equal(bits(sf), bits(cols.static_f)), "static_f"
    assert np.array_equal(si, cols.static_i), "static_i (IST/ICE derived from the table types)"


def test_state_round_trip(tmp_path, ref_params):
    cols = cases.make_columns(32, "mixed", ref_params, seed=5)
    grid = grid_for(cols)
    p = str(tmp_path / "init.nc")
    t = datetime.datetime(2000, 3, 1, 6)
    ncio.write_state(p, grid, cols.state, cols.isnow, t, step=17)
    st, isn, t2, step = ncio.read_state(p, grid)
    assert np.array_equal(bits(st), bits(cols.state)) and np.array_equal(isn, cols.isnow)
    assert t2 == t and step == 17
    st64 = cols.state.astype(np.float64)
    ncio.write_state(p, grid, st64, cols.isnow, t)
    assert np.array_equal(bits(ncio.read_state(p, grid, np.float64)[0]), bits(st64))


def test_ldasin_round_trip_and_derived_fields(tmp_path, ref_params):
    cols = cases.make_columns(32, "mixed", ref_params, seed=6, julian=0.0)
    grid = grid_for(cols)
    f = cases.forcing_step(cols, 0.25, 366, 0, seed=1)
    d = tmp_path / "ldasin"
    d.mkdir()
    ncio.write_ldasin(ncio.ldasin_path(str(d), T0), grid, f, T0, extras=True)
    prov = ncio.LdasinForcing(str(d), grid, T0, datetime.timedelta(hours=1))
    got = prov(0, T0)
    assert np.array_equal(bits(got), bits(f)), "LDASIN with extras reproduces the slice"
    # held over the input interval: 00:45 reads the 00:00 file
    assert prov.input_time(T0 + datetime.timedelta(minutes=45)) == T0
    assert np.array_equal(bits(prov(3, T0 + datetime.timedelta(minutes=45))[:9]), bits(f[:9]))
    # standard HRLDAS file (no extras): COSZ from the grid at the step time, CO2/O2 from PSFC
    ncio.write_ldasin(ncio.ldasin_path(str(d), T0), grid, f, T0, extras=False)
    t = T0 + datetime.timedelta(minutes=30)
    g = ncio.LdasinForcing(str(d), grid, T0, datetime.timedelta(hours=1))(2, t)
    cz = timeman.cosz(grid.lat_rad, grid.lon_rad, timeman.julian(t), 366).astype(np.float32)
    assert np.array_equal(bits(g[L.FORCING.index("COSZ")]), bits(cz))
    psfc = f[L.FORCING.index("PSFC")].astype(np.float64)
    assert np.array_equal(bits(g[L.FORCING.index("CO2AIR")]), bits(np.float32(395e-6 * psfc)))
    assert np.array_equal(g[L.FORCING.index("SFCPRS")], f[L.FORCING.index("PSFC")])
    # the LDASIN block the engine expands on the device (nmp_forcing_from_ldasin):
    # the file's variables + the same COSZ; restated here as the kernel forms
    # the fields, it gives the host reader's 12 bit for bit
    prov2 = ncio.LdasinForcing(str(d), grid, T0, datetime.timedelta(hours=1))
    raw = prov2.raw(2, t)
    assert raw.dtype == np.float32 and raw.shape == (L.NLDASIN, 32)
    R = {v: raw[i] for i, v in enumerate(L.LDASIN)}
    x = {"SFCTMP": R["T2D"], "SFCPRS": R["PSFC"], "PSFC": R["PSFC"], "UU": R["U2D"],
         "VV": R["V2D"], "Q2": R["Q2D"], "SOLDN": R["SWDOWN"], "LWDN": R["LWDOWN"],
         "PRCP": R["RAINRATE"], "COSZ": R["COSZ"],
         "CO2AIR": np.float32(395.0e-6 * R["PSFC"].astype(np.float64)),
         "O2AIR": np.float32(0.209 * R["PSFC"].astype(np.float64))}
    assert np.array_equal(bits(np.stack([x[k] for k in L.FORCING])), bits(g))
    # the once-per-interval block (device COSZ): the 8 file variables as in
    # raw, the COSZ row left alone (the file has none), and the geometry whose
    # COSZ expression, restated from solar_terms, is timeman.cosz's bit for bit
    blk = np.full((L.NLDASIN, 32), -7.0, np.float32)
    assert prov2.block(t, out=blk) is blk and not prov2.file_cosz(t)
    ci = L.LDASIN.index("COSZ")
    assert np.array_equal(bits(np.delete(blk, ci, 0)), bits(np.delete(raw, ci, 0)))
    assert (blk[ci] == -7.0).all()
    geo = prov2.geo()
    assert geo.dtype == np.float64 and geo.shape == (3, 32)
    sd, cd, ha0 = timeman.solar_terms(timeman.julian(t), 366)
    cz_geo = geo[0] * sd + (geo[1] * cd) * np.cos((ha0 + geo[2]) - np.pi)
    assert np.array_equal(bits(cz_geo.astype(np.float32)), bits(cz))
    # the device-ingest form: the file's own big-endian fp32 grids, every grid
    # point, whose land points in prov2's column order are the block's rows
    assert prov2.ingestible(t) and prov2.variables(t) == frozenset(L.LDASIN[:-1])
    gr = prov2.grid_raw(t)
    assert gr.dtype == np.dtype(">f4") and gr.shape == (L.NLDASIN - 1, 40)
    assert np.array_equal(bits(gr[:, prov2.point()].astype(np.float32)),
                          bits(np.delete(raw, ci, 0)))
    # a file holding a variable in fp64 is not ingestible (the driver then
    # builds the block on the host)
    from scipy.io import netcdf_file
    p64 = ncio.ldasin_path(str(d), T0 + datetime.timedelta(hours=1))
    ncio.write_ldasin(p64, grid, f, T0, extras=False)
    with netcdf_file(p64, "a") as nc:
        v = nc.createVariable("T2D_", "f8", ("Time", "south_north", "west_east"))
        v[0] = np.zeros(grid.shape)
    prov3 = ncio.LdasinForcing(str(d), grid, T0, datetime.timedelta(hours=1))
    assert prov3.ingestible(T0 + datetime.timedelta(hours=1))   # extra variables do not matter
    ncio.write_ldasin(p64, grid, f, T0, extras=False)
    with netcdf_file(p64, "r") as nc:
        vs = {k: np.array(nc.variables[k][0]) for k in nc.variables}
    with netcdf_file(p64, "w") as nc:
        nc.createDimension("Time", None)
        nc.createDimension("south_north", 5)
        nc.createDimension("west_east", 8)
        for k, a in vs.items():
            v = nc.createVariable(k, "f8" if k == "T2D" else "f4", ("Time", "south_north",
                                                                     "west_east"))
            v[0] = a
    prov4 = ncio.LdasinForcing(str(d), grid, T0, datetime.timedelta(hours=1))
    assert not prov4.ingestible(T0 + datetime.timedelta(hours=1))
    # a file with its own CO2AIR / O2AIR has no block form
    ncio.write_ldasin(ncio.ldasin_path(str(d), T0), grid, f, T0, extras=("CO2AIR",))
    assert ncio.LdasinForcing(str(d), grid, T0, datetime.timedelta(hours=1)).raw(0, T0) is None
    with pytest.raises(FileNotFoundError):
        prov(8, T0 + datetime.timedelta(hours=2))


def test_ldasout_round_trip(tmp_path, ref_params):
    cols = cases.make_columns(32, "mixed", ref_params, seed=7)
    grid = grid_for(cols)
    diag = np.random.default_rng(0).normal(size=(L.NDIAG_OUT, 32)).astype(np.float32)
    p = ncio.ldasout_path(str(tmp_path), T0)
    ncio.write_ldasout(p, grid, diag, T0)
    assert p.endswith("2000010100.LDASOUT_DOMAIN1")
    assert np.array_equal(bits(ncio.read_ldasout(p, grid)), bits(diag))
    raw = ncio.read_ldasin(p)
    assert (raw["FSA"][~grid.mask] == ncio.FILL).all()
    # engine-ordered fluxes (column j = land point perm[j]), scattered on a
    # pool, fp32 and fp64: the same file contents as the grid-ordered write
    from concurrent.futures import ThreadPoolExecutor
    perm = np.random.default_rng(1).permutation(32)
    for dt in (np.float32, np.float64):
        d = diag.astype(dt)
        q = str(tmp_path / f"perm_{np.dtype(dt).itemsize}.nc")
        with ThreadPoolExecutor(3) as pool:
            ncio.write_ldasout(q, grid, d[:, perm], T0, cols=perm, pool=pool)
        got = ncio.read_ldasout(q, grid)
        assert got.dtype == dt and np.array_equal(bits(got), bits(d))
        assert (ncio.read_ldasin(q)["FSH"][~grid.mask] == ncio.FILL).all()


def test_trajectory_fixture_fits_the_files(tmp_path):
    """The inputs of the reference trajectory survive the netCDF layouts bit for
    bit (what tests/test_gpu_driver.py::test_driver_from_netcdf_files runs)."""
    g = load("traj_casenml.npz")
    cols = cases.ColumnSet(g["static_f"], g["static_i"], g["state0"], g["isnow0"], *([None] * 7))
    grid = grid_for(cols)
    p = str(tmp_path / "geo.nc")
    ncio.write_static(p, cols, grid)
    _, sf, si = ncio.read_static(p, load_params_dict(), T0)
    assert np.array_equal(bits(sf), bits(g["static_f"])) and np.array_equal(si, g["static_i"])


def load_params_dict():
    from noahmp_amd.params import Params
    return Params.builtin().as_dict()


def test_ldasout_from_grids_is_the_same_file(tmp_path, ref_params):
    """ncio.write_ldasout_grids (the header built from the netCDF-3 layout
    plus the fluxes already on the file's big-endian grids, as
    nmp_ldasout_grid forms them on the device) writes the very bytes of
    write_ldasout (scipy's netcdf writer) -- fp32 and fp64, a grid with ocean
    points, two valid times."""
    cols = cases.make_columns(32, "mixed", ref_params, seed=8)
    grid = grid_for(cols)
    for dt in (np.float32, np.float64):
        diag = np.random.default_rng(2).normal(size=(L.NDIAG_OUT, 32)).astype(dt)
        full = np.stack([grid.scatter(diag[i], np.asarray(ncio.FILL, dt)).reshape(-1)
                         for i in range(L.NDIAG_OUT)]).astype(np.dtype(dt).newbyteorder(">"))
        for t in (T0, T0 + datetime.timedelta(hours=3, minutes=30)):
            a, b = str(tmp_path / "a.nc"), str(tmp_path / "b.nc")
            ncio.write_ldasout(a, grid, diag, t)
            ncio.write_ldasout_grids(b, grid, full, t)
            assert open(a, "rb").read() == open(b, "rb").read()
            assert np.array_equal(bits(ncio.read_ldasout(b, grid)), bits(diag))


def test_ldasout_header_refuses_past_classic_offsets():
    """A grid whose 16 fp64 fluxes pass the classic format's signed 32-bit
    offsets (2 GiB) is refused rather than written with wrapped offsets."""
    big = ncio.Grid(np.zeros((1, 1)), np.zeros((1, 1)), np.ones((1, 1), bool))
    big.shape = (4096, 4096)          # 16.8 M points: 16 x 8 B x 16.8 M = 2.1 GB
    with pytest.raises(ValueError, match="2 GiB"):
        ncio.ldasout_header(big, "f8", T0)
    assert len(ncio.ldasout_header(big, "f4", T0)) > 0   # 1.07 GB fits
