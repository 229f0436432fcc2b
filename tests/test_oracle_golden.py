"""Pin the C restatement (oracle/noahmp_oracle.c) to the reference Fortran.

Every fixture in tests/golden/ was produced by the reference noahmp_sflx
(core/module_noahmp_func.f90:66-476) compiled by oracle/Makefile; see
tests/golden/make_golden.py.  The bar here is BIT-EXACT: same fp32 operation
order, same libm, no contraction.
"""
import numpy as np
import pytest

from golden_io import (as_ref_status, bit_equal, fixture_params, fixture_tags, load, load_params,
                       single_names)
from noahmp_amd import layout as L


@pytest.mark.parametrize("name", single_names())
def test_single_call_bit_exact(oracle_port, name):
    g = load(f"single_{name}.npz")
    P = fixture_params(g)
    st, isn, dg, status = oracle_port.step(P, tuple(g["options"]), g["zsoil"], float(g["dt"]),
                                           int(g["yearlen"]), float(g["julian"]), g["state0"],
                                           g["isnow0"], g["static_f"], g["static_i"], g["forcing"])
    assert np.array_equal(as_ref_status(status), g["status"])
    assert np.array_equal(isn, g["isnow1"])
    bad = ~bit_equal(st, g["state1"])
    assert not bad.any(), list(np.nonzero(bad.any(1))[0])
    bad = ~bit_equal(dg, g["diag"])
    assert not bad.any(), [L.DIAG_FULL[f] for f in np.nonzero(bad.any(1))[0]]


@pytest.mark.parametrize("name", ["casenml", "snow", "combo_a"])
def test_trajectory_bit_exact(oracle_port, name):
    g = load(f"traj_{name}.npz")
    P = load_params()
    opts, dt, ylen, ke = tuple(g["options"]), float(g["dt"]), int(g["yearlen"]), int(g["keep_every"])
    st, isn = g["state0"], g["isnow0"]
    nsteps = g["forcing"].shape[0]
    k = 0
    for s in range(nsteps):
        jul = float(g["julian0"]) + s * dt / 86400.0
        st, isn, dg, status = oracle_port.step(P, opts, g["zsoil"], dt, ylen, jul, st, isn,
                                               g["static_f"], g["static_i"], g["forcing"][s])
        if (s + 1) % ke == 0 or s == nsteps - 1:
            assert bit_equal(st, g["states"][k]).all(), f"state diverged at step {s}"
            assert np.array_equal(isn, g["isnows"][k]), s
            assert bit_equal(dg, g["diags"][k]).all(), f"diag diverged at step {s}"
            assert np.array_equal(as_ref_status(status), g["statuses"][k]), s
            k += 1
    assert k == g["states"].shape[0]


def test_fixture_coverage():
    """The fixtures exercise the regimes the kernels branch on."""
    g = load("single_casenml_mixed.npz")
    isn = g["isnow0"]
    assert set(np.unique(isn)) == {-3, -2, -1, 0}
    assert (g["forcing"][L.FORCING.index("COSZ")] <= 0).any()
    assert (g["forcing"][L.FORCING.index("COSZ")] > 0).any()
    c = load("single_casenml_conus.npz")
    assert {1, 2} == set(np.unique(c["static_i"][L.STATIC_I.index("IST")]))
    assert {0, 1} == set(np.unique(c["static_i"][L.STATIC_I.index("ICE")]))
    z = load("single_fatal.npz")
    assert (z["status"] != 0).any() and (z["status"] == 0).any()
    opts = {tuple(load(f"single_{n}.npz")["options"]) for n in single_names()}
    for k, name in enumerate(L.OPTION_NAMES):
        lo, hi = L.OPTION_RANGES[name]
        assert {o[k] for o in opts} == set(range(lo, hi + 1)), name
    tags = {fixture_tags(load(f"single_{n}.npz")) for n in single_names()}
    assert {("STAS", "USGS"), ("STAS-RUC", "USGS"), ("STAS", "MODIFIED_IGBP_MODIS_NOAH"),
            ("STAS-RUC", "MODIFIED_IGBP_MODIS_NOAH")} <= tags
    combos = [o for o in opts if sum(v != d for v, d in zip(o, L.options_tuple(L.CASE_NML_OPTIONS))) >= 3]
    assert len(combos) >= 3, "option-combination fixtures"
    t = load("traj_snow.npz")
    assert (t["isnows"] != t["isnows"][:1]).any(), "snow trajectory never changes layering"


def test_fp64_restatement_tracks_fp32(oracle_port):
    """The fp64 restatement (engine precision 8 oracle) stays near the fp32 reference."""
    g = load("single_casenml_conus.npz")
    P = load_params()
    st, isn, dg, status = oracle_port.step(P, tuple(g["options"]), g["zsoil"], float(g["dt"]),
                                           int(g["yearlen"]), float(g["julian"]), g["state0"],
                                           g["isnow0"], g["static_f"], g["static_i"], g["forcing"],
                                           precision=8)
    same = isn == g["isnow1"]
    assert same.mean() > 0.99
    stc = L.s("STC")
    d = np.abs(st[stc][:, same] - g["state1"][stc][:, same])
    assert np.nanpercentile(d, 99) < 1e-2


@pytest.mark.parametrize("name", single_names())
def test_cr_math_restatement_meets_parity_bar(oracle_port, name):
    """The same fp32 algorithm with correctly rounded libm (the engine's default
    math) meets the GPU parity bar against the reference: the bar's residual
    is glibc float-libm rounding, not algorithm."""
    from golden_io import parity_vs_reference
    g = load(f"single_{name}.npz")
    out = oracle_port.step(fixture_params(g), tuple(g["options"]), g["zsoil"], float(g["dt"]),
                           int(g["yearlen"]), float(g["julian"]), g["state0"], g["isnow0"],
                           g["static_f"], g["static_i"], g["forcing"], precision="cr")
    r, msg = parity_vs_reference(*out, g)
    assert not msg, msg
    assert r["exact"] > 0.7
