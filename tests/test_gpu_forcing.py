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
