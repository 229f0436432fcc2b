"""Device forcing generator (nmp_forcing_synth, csrc/forcing.hip) against its
numpy restatement (tests/forcing_twin.py), and its invariances: stateless in
(seed, step, global column), so column ranges and ranks reproduce one launch."""
import numpy as np
import pytest
import torch

import noahmp_pkg  # noqa: F401
from noahmp_amd import cases, layout as L

DEV = "cuda:0"


def test_forcing_twin_on_cpu_is_physical():
    """(CPU) the restatement yields physical forcing for the global grid kind."""
    from forcing_twin import synth
    from noahmp_amd.params import Params
    cols = cases.make_columns(4096, "global", Params.builtin().as_dict(), seed=2, first=500_000)
    f = synth(cases.climate(cols), 180.25, 366, 77, 5, 500_000)
    F = L.FORCING.index
    assert np.isfinite(f).all()
    assert (f[F("SOLDN")] >= 0).all() and (np.abs(f[F("COSZ")]) <= 1).all()
    assert (f[F("PRCP")] >= 0).all() and 0 < (f[F("PRCP")] > 0).mean() < 0.5
    assert (f[F("Q2")] > 0).all() and (f[F("LWDN")] > 100).all()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [4, 8])
def test_device_forcing_matches_restatement(engine_lib, precision):
    from forcing_twin import synth
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    dt = torch.float32 if precision == 4 else torch.float64
    npdt = np.float32 if precision == 4 else np.float64
    n = 100_003
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=4, julian=200.0)
    clim = torch.as_tensor(cases.climate(cols), device=DEV).to(dt).contiguous()
    eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=precision)
    out = torch.zeros((L.NFORCING, n), dtype=dt, device=DEV)
    for step, jul in ((0, 200.0), (37, 200.77), (8783, 365.96)):
        eng.forcing_synth(clim, jul, 366, 1234, step, out, first_col=10_000)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        want = synth(clim.cpu().numpy(), jul, 366, 1234, step, 10_000, npdt)
        F = L.FORCING.index
        # the rain decision is an exact comparison of hash bits: identical
        assert np.array_equal(got[F("PRCP")] > 0, want[F("PRCP")] > 0)
        # ocml vs glibc double libm differ by <= 1 ulp of double: after the
        # rounding to fp32 a few ulp at most; in fp64 the ulp survives, and
        # sums that cancel (COSZ near the terminator) amplify it relatively
        rtol, atol = (4e-6, 4e-8) if precision == 4 else (1e-10, 1e-12)
        np.testing.assert_allclose(got, want, rtol=rtol, atol=atol)
    eng.close()


@pytest.mark.gpu
def test_device_forcing_is_stateless_over_ranges(engine_lib):
    """Generating column ranges separately (as StreamShards ranges or ranks do,
    with their global first column) gives exactly the one-launch result."""
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    n = 50_000
    cols = cases.make_columns(n, "global", Params.builtin().as_dict(), seed=3)
    clim = torch.as_tensor(cases.climate(cols, np.float32), device=DEV)
    eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0)
    a = torch.zeros((L.NFORCING, n), device=DEV)
    b = torch.zeros_like(a)
    eng.forcing_synth(clim, 10.5, 365, 9, 3, a)
    for lo, hi in ((0, 12_345), (12_345, 40_000), (40_000, n)):
        eng.forcing_synth(clim, 10.5, 365, 9, 3, b, cols=(lo, hi))
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [4, 8])
def test_forcing_from_ldasin_equals_host_reader(engine_lib, precision):
    """nmp_forcing_from_ldasin: the 12 forcing fields the engine forms from the
    uploaded LDASIN block (8 file variables + COSZ, fp32) are, bit for bit,
    the fields the host reader builds (ncio.LdasinForcing.__call__: SFCPRS =
    PSFC, CO2AIR / O2AIR = 395e-6 / 0.209 PSFC in double rounded to fp32), then
    widened to the engine precision; column ranges give the one-launch result."""
    from noahmp_amd import ncio
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    dt = torch.float32 if precision == 4 else torch.float64
    n = 70_001
    cols = cases.make_columns(n, "conus", Params.builtin().as_dict(), seed=6, julian=100.0)
    f = cases.forcing_step(cols, 100.25, 366, 3, seed=6)
    # pressures the fp32 file holds (a double product of an fp32 pressure
    # rounds differently from one of the generator's double pressure)
    fl = {var: f[L.FORCING.index(fld)] for fld, var in ncio.LDASIN_MAP.items()}
    fl["COSZ"] = f[L.FORCING.index("COSZ")]
    raw = np.stack([fl[v] for v in L.LDASIN]).astype(np.float32)
    want = np.empty((L.NFORCING, n), np.float32)
    for fld, var in ncio.LDASIN_MAP.items():
        want[L.FORCING.index(fld)] = fl[var]
    want[L.FORCING.index("COSZ")] = fl["COSZ"]
    psfc = fl["PSFC"].astype(np.float64)
    want[L.FORCING.index("CO2AIR")] = 395.0e-6 * psfc
    want[L.FORCING.index("O2AIR")] = 0.209 * psfc
    want = want.astype(np.float32 if precision == 4 else np.float64)
    eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=precision)
    r = torch.as_tensor(raw, device=DEV)
    a = torch.zeros((L.NFORCING, n), dtype=dt, device=DEV)
    b = torch.full_like(a, float("nan"))
    eng.forcing_from_ldasin(r, a)
    for lo, hi in ((0, 4_097), (4_097, 50_000), (50_000, n)):
        eng.forcing_from_ldasin(r, b, cols=(lo, hi))
    torch.cuda.synchronize()
    iv = torch.int32 if precision == 4 else torch.int64
    got = a.cpu().numpy()
    assert np.array_equal(got.view(np.int32 if precision == 4 else np.int64),
                          want.view(np.int32 if precision == 4 else np.int64))
    assert torch.equal(a.view(iv), b.view(iv))
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [4, 8])
def test_forcing_from_ldasin_geo_device_cosz(engine_lib, precision):
    """nmp_forcing_from_ldasin_geo: COSZ formed on the device from the columns'
    (sin lat, cos lat, lon) and the step's solar terms, in timeman.cosz's
    expression and order, rounded to fp32.  Over 1,000,003 columns spread over
    the globe and 8 times of day through a year, it equals the host's
    (numpy double cosine) on at least 99.999 % of the column-steps and is never
    more than 1 fp32 ulp away; the block's COSZ row is not read; the other 11
    fields are nmp_forcing_from_ldasin's, bit for bit; column ranges give the
    one-launch result."""
    from noahmp_amd import timeman
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    dt = torch.float32 if precision == 4 else torch.float64
    n = 1_000_003
    rng = np.random.default_rng(11)
    lat = np.radians(rng.uniform(-89.9, 89.9, n))
    lon = np.radians(rng.uniform(-180.0, 180.0, n))
    geo = torch.as_tensor(np.stack([np.sin(lat), np.cos(lat), lon]), device=DEV)
    raw = rng.uniform(1.0, 2.0, (L.NLDASIN, n)).astype(np.float32)
    raw[L.LDASIN.index("PSFC")] *= 5.0e4
    r = torch.as_tensor(raw, device=DEV)
    eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=precision)
    a = torch.zeros((L.NFORCING, n), dtype=dt, device=DEV)
    b = torch.full_like(a, float("nan"))
    plain = torch.zeros_like(a)
    eng.forcing_from_ldasin(r, plain)
    ci = L.FORCING.index("COSZ")
    mism, total = 0, 0
    for jul in (1.0, 45.3125, 100.5, 172.75, 200.0625, 266.875, 300.4375, 365.9583):
        solar = timeman.solar_terms(jul, 366)
        eng.forcing_from_ldasin(r, a, geo=geo, solar=solar)
        for lo, hi in ((0, 65_537), (65_537, 700_000), (700_000, n)):
            eng.forcing_from_ldasin(r, b, cols=(lo, hi), geo=geo, solar=solar)
        torch.cuda.synchronize()
        iv = torch.int32 if precision == 4 else torch.int64
        assert torch.equal(a.view(iv), b.view(iv))
        keep = [i for i in range(L.NFORCING) if i != ci]
        assert torch.equal(a[keep].view(iv), plain[keep].view(iv))
        got = a[ci].cpu().numpy().astype(np.float32)
        want = timeman.cosz(lat, lon, jul, 366).astype(np.float32)
        ulps = np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
        # (same-sign values: the int distance is the ulp distance; |COSZ| <= 1)
        same = np.sign(got) == np.sign(want)
        assert (ulps[same] <= 1).all() and (got[~same] == want[~same]).all()
        mism += int((ulps != 0).sum())
        total += n
    print(f"device COSZ: {mism} of {total} column-steps differ from numpy's by 1 fp32 ulp")
    assert mism <= 1e-5 * total
    eng.close()


@pytest.mark.gpu
def test_ldasin_ingest_equals_host_block(engine_lib, tmp_path):
    """nmp_ldasin_ingest: an LDASIN file's bytes as stored (ncio grid_raw:
    big-endian grids, ocean points included) selected, ordered and
    byte-swapped on the device give the host block's 8 rows (ncio block: the
    land points in the engine's column order) bit for bit; the COSZ row is not
    written; a point outside the grid gives NaN rows (no out-of-bounds load)."""
    import datetime
    from noahmp_amd import ncio
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    ny, nx = 40, 64
    rng = np.random.default_rng(3)
    mask = rng.uniform(size=(ny, nx)) < 0.6
    lat = np.broadcast_to(np.linspace(20.0, 50.0, ny)[:, None], (ny, nx))
    lon = np.broadcast_to(np.linspace(-120.0, -70.0, nx)[None, :], (ny, nx))
    grid = ncio.Grid(lat, lon, mask)
    n = grid.n
    cols = cases.make_columns(n, "conus", Params.builtin().as_dict(), seed=2, julian=100.0)
    t0 = datetime.datetime(2000, 4, 10)
    d = tmp_path / "ldasin"
    d.mkdir()
    ncio.write_ldasin(ncio.ldasin_path(str(d), t0), grid,
                      cases.forcing_step(cols, 100.0, 366, 0, seed=2), t0, extras=False)
    perm = rng.permutation(n)
    fr = ncio.LdasinForcing(str(d), grid, t0, datetime.timedelta(hours=1), cols=perm, threads=3)
    want = fr.block(t0, out=np.zeros((L.NLDASIN, n), np.float32))
    g = fr.grid_raw(t0, out=np.empty((L.NLDASIN - 1, ny * nx), np.int32))
    point = fr.point()
    point[5] = ny * nx          # one column outside the grid
    eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=4)
    out = torch.full((L.NLDASIN, n), -3.0, dtype=torch.float32, device=DEV)
    eng.ldasin_ingest(torch.as_tensor(g, device=DEV), torch.as_tensor(point, device=DEV), out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ci = L.LDASIN.index("COSZ")
    ok = np.ones(n, bool)
    ok[5] = False
    assert np.array_equal(np.delete(got, ci, 0)[:, ok].view(np.int32),
                          np.delete(want, ci, 0)[:, ok].view(np.int32))
    assert np.isnan(np.delete(got, ci, 0)[:, 5]).all()
    assert (got[ci] == -3.0).all()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [4, 8])
def test_ldasout_grid_equals_host_scatter(engine_lib, precision):
    """nmp_ldasout_grid: 16 fluxes of n columns (engine precision) laid on
    the file's grids in its byte order on the device equal the host's
    grid.scatter with FILL, converted to big-endian, bit for bit; a point
    outside the grid is skipped."""
    from noahmp_amd import ncio
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    dt = np.float32 if precision == 4 else np.float64
    ny, nx = 37, 53
    rng = np.random.default_rng(4)
    mask = rng.uniform(size=(ny, nx)) < 0.7
    grid = ncio.Grid(np.zeros((ny, nx)), np.zeros((ny, nx)), mask)
    n = grid.n
    diag = rng.normal(size=(L.NDIAG_OUT, n)).astype(dt)
    perm = rng.permutation(n)
    point = np.asarray(grid.index)[perm].astype(np.int32)
    want = np.stack([grid.scatter(diag[i], np.asarray(ncio.FILL, dt)).reshape(-1)
                     for i in range(L.NDIAG_OUT)]).astype(np.dtype(dt).newbyteorder(">"))
    eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=precision)
    iv = torch.int32 if precision == 4 else torch.int64
    out = torch.zeros((L.NDIAG_OUT, ny * nx), dtype=iv, device=DEV)
    d = torch.as_tensor(np.ascontiguousarray(diag[:, perm]), device=DEV)
    bad = point.copy()
    bad[7] = -1
    eng.ldasout_grid(d, torch.as_tensor(point, device=DEV), out, float(ncio.FILL))
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(want.dtype)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    eng.ldasout_grid(d, torch.as_tensor(bad, device=DEV), out, float(ncio.FILL))
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(want.dtype)
    skip = point[7]
    want[:, skip] = np.asarray(ncio.FILL, dt)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    eng.close()


@pytest.mark.gpu
def test_ldasin_ldasout_entries_reject_bad_arguments(engine_lib):
    """The file-format entries check their sizes before launching: a leading
    dimension below ncol, an empty or oversized grid, too many fields, or a
    missing pointer return NMP_E_ARG and leave the output untouched; zero
    columns is a no-op."""
    import ctypes as C
    from noahmp_amd.engine import Engine, _ptr
    from noahmp_amd.params import Params
    eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=4)
    lib, h = eng._lib, eng._h
    n, npts = 64, 100
    g = torch.zeros((L.NLDASIN - 1, npts), dtype=torch.int32, device=DEV)
    pt = torch.arange(n, dtype=torch.int32, device=DEV)
    blk = torch.full((L.NLDASIN, n), 7.0, device=DEV)
    diag = torch.zeros((L.NDIAG_OUT, n), device=DEV)
    out = torch.full((L.NDIAG_OUT, npts), 5, dtype=torch.int32, device=DEV)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    E_ARG = -1
    assert lib.nmp_ldasin_ingest(h, n, n - 1, npts, _ptr(g), _ptr(pt), _ptr(blk), s) == E_ARG
    assert lib.nmp_ldasin_ingest(h, n, n, 0, _ptr(g), _ptr(pt), _ptr(blk), s) == E_ARG
    assert lib.nmp_ldasin_ingest(h, n, n, 1 << 29, _ptr(g), _ptr(pt), _ptr(blk), s) == E_ARG
    assert lib.nmp_ldasin_ingest(h, n, n, npts, None, _ptr(pt), _ptr(blk), s) == E_ARG
    assert lib.nmp_ldasin_ingest(h, 0, n, npts, _ptr(g), _ptr(pt), _ptr(blk), s) == 0
    assert lib.nmp_ldasout_grid(h, n, n, npts, L.NDIAG_FULL + 1, _ptr(diag), _ptr(pt), -9999.0,
                                _ptr(out), s) == E_ARG
    assert lib.nmp_ldasout_grid(h, n, n - 1, npts, 16, _ptr(diag), _ptr(pt), -9999.0, _ptr(out),
                                s) == E_ARG
    assert lib.nmp_ldasout_grid(h, n, n, npts, 16, None, _ptr(pt), -9999.0, _ptr(out), s) == E_ARG
    assert lib.nmp_forcing_from_ldasin_geo(h, n, n, _ptr(blk), None, 0.0, 1.0, 0.0,
                                           _ptr(diag), s) == E_ARG
    torch.cuda.synchronize()
    assert (blk == 7.0).all() and (out == 5).all()
    eng.close()
