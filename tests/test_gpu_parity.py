"""HIP engine parity against the reference (golden fixtures) and the oracle.

Everything here calls the engine through the C ABI (noahmp_amd.engine ->
libnoahmp_engine.so).  Two tiers:

1. GPU (default "ref" math: glibc's float libm restated bit-exactly, see
   csrc/glibc_math.h and tests/test_glibc_math.py) vs the reference fixtures:
   bit-identical on every column of every fixture -- state, all 58 outputs,
   ISNOW, status -- and along both trajectories (96 case.nml steps, 480 snow
   steps through layer combine/divide).
2. GPU vs the reference Fortran fixtures: golden_io.parity_vs_reference --
   >= 97 % of columns within the SURVEY 8c tolerance (states |d| <= 1e-4 +
   1e-5|ref|, fluxes |d| <= 1e-2 + 1e-4|ref|), >= 99.5 % of the remaining
   columns within the loose envelope (1e-3 / 2e-2 rel), <= 2 % ISNOW or
   fatal-status flips.  Those residuals are glibc float-libm ulps (tanhf /
   atanf are not correctly rounded) amplified by Newton iteration counts; the
   same bar is met by the CR oracle on the CPU (test_oracle_golden.py).

fp64 engine vs the fp64 restatement: |d| <= 1e-9 (1 + |ref|) on >= 99 % of
columns (ocml vs glibc double libm ulps).
"""
import dataclasses

import numpy as np
import pytest
import torch

from golden_io import (FP64_POOLED_FRAC, FP64_TOL_FRAC, as_ref_status, bit_equal,
                       check_fp64_trajectory_step, close, column_mismatch, fixture_tags, load,
                       load_params, parity_fp64_vs_reference, parity_vs_reference, single_names)
from noahmp_amd import cases, layout as L

pytestmark = pytest.mark.gpu

STATE_NAMES = [f"{n}[{k}]" if w > 1 else n for n, w in L.STATE_FIELDS for k in range(w)]
DEV = "cuda:0"
# Both occupancy instantiations of the step kernel (nmp_set_launch_variant):
# "small" is what the fixture sizes select by themselves (half occupancy),
# "full" the 4-waves/SIMD fp32 / 2-waves fp64 kernel every production-size
# launch runs.  Register allocation differs between them, so each is pinned
# to the reference on its own ("What's weak" 1).
VARIANTS = ["small", "full"]
VARIANTS32 = VARIANTS


@pytest.fixture(scope="module")
def engines(engine_lib):
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    cache, tables = {}, {}

    def get(options, precision=4, math="ref", tags=("STAS", "USGS"), variant="auto"):
        key = (tuple(int(x) for x in options), precision, math, tuple(tags), variant)
        if key not in cache:
            if tags not in tables:
                tables[tags] = Params.builtin(*tags)
            cache[key] = Engine(tables[tags], dict(zip(L.OPTION_NAMES, key[0])), device=0,
                                precision=precision, math=math)
            assert cache[key].launch_variant(variant) == variant
        return cache[key]
    return get


def run_single(eng, g, dtype=torch.float32):
    from noahmp_amd.engine import ColumnState
    cols = cases.ColumnSet(g["static_f"], g["static_i"], g["state0"], g["isnow0"],
                           *([None] * 7))
    cs = ColumnState.from_host(cols, DEV, dtype)
    f = torch.as_tensor(g["forcing"], device=DEV).to(dtype).contiguous()
    diag = torch.zeros((L.NDIAG_FULL, cs.ncol), dtype=dtype, device=DEV)
    eng.step(cs, f, g["zsoil"], float(g["dt"]), float(g["julian"]), int(g["yearlen"]), diag,
             L.DIAG_FULL_LEVEL)
    torch.cuda.synchronize()
    return (cs.state.cpu().numpy(), cs.isnow.cpu().numpy(), diag.cpu().numpy(),
            cs.status.cpu().numpy())


def oracle_single(port, g, precision):
    return port.step(load_params(), tuple(g["options"]), g["zsoil"], float(g["dt"]),
                     int(g["yearlen"]), float(g["julian"]), g["state0"], g["isnow0"],
                     g["static_f"], g["static_i"], g["forcing"], precision=precision)


@pytest.mark.parametrize("name", single_names())
def test_single_call_vs_reference(engines, name):
    g = load(f"single_{name}.npz")
    r, msg = parity_vs_reference(*run_single(engines(g["options"], tags=fixture_tags(g)), g), g)
    print(name, r)
    assert not msg, f"{name}: {msg}"


@pytest.mark.parametrize("variant", VARIANTS32)
@pytest.mark.parametrize("name", single_names())
def test_single_call_bit_exact_vs_reference(engines, name, variant):
    """Default ("ref") math = glibc's float libm restated bit-exactly
    (csrc/glibc_math.h), so the kernel must reproduce the reference Fortran
    bit for bit: every state field, every one of the 58 outputs, ISNOW, status
    -- in both occupancy instantiations of every option-set kernel the
    fixture's options select (set 1, set 2 or the run-time-options set 0)."""
    g = load(f"single_{name}.npz")
    st, isn, dg, status = run_single(
        engines(g["options"], tags=fixture_tags(g), variant=variant), g)
    exact = bit_equal(st, g["state1"]).all(0) & bit_equal(dg, g["diag"]).all(0) & \
        (isn == g["isnow1"]) & (as_ref_status(status) == g["status"])
    _, rep_s = column_mismatch(st, g["state1"], 0, 0, STATE_NAMES)
    _, rep_d = column_mismatch(dg, g["diag"], 0, 0, L.DIAG_FULL)
    print(name, "bit-exact columns", exact.mean())
    assert exact.all(), \
        f"{name}: {(~exact).sum()} columns differ from the reference: " + "; ".join(
            rep_s[:8] + rep_d[:8])


@pytest.mark.parametrize("name", ["casenml_mixed", "casenml_conus", "veg2", "run3", "frz2",
                                  "sfc2", "fatal"])
def test_single_call_fp64_vs_fp64_oracle(engines, oracle_port, name):
    g = load(f"single_{name}.npz")
    est, eisn, edg, estat = oracle_single(oracle_port, g, 8)
    st, isn, dg, status = run_single(engines(g["options"], 8), g, torch.float64)
    ok = close(st, est, 1e-9, 1e-9).all(0) & close(dg, edg, 1e-9, 1e-9).all(0) & \
        (isn == eisn) & (status == estat)
    _, rep_s = column_mismatch(st, est, 1e-9, 1e-9, STATE_NAMES)
    _, rep_d = column_mismatch(dg, edg, 1e-9, 1e-9, L.DIAG_FULL)
    assert ok.mean() >= 0.99 or (~ok).sum() <= 1, "; ".join(rep_s[:8] + rep_d[:8])


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", single_names())
def test_single_call_fp64_vs_reference(engines, name, variant):
    """fp64 engine vs the fp32 REFERENCE fixtures at SURVEY 8c's x10 bar on all
    56 state values and all 58 outputs (golden_io.parity_fp64_vs_reference):
    >= 97 % of non-tie columns inside the bar, at most one column outside the
    loop-exit envelope.  The CPU twin of this test
    (test_oracle_golden.py::test_fp64_restatement_vs_fp32_reference) shows the
    misses are Newton/bisection loops exiting on another iteration in fp64."""
    g = load(f"single_{name}.npz")
    out = run_single(engines(g["options"], 8, tags=fixture_tags(g), variant=variant), g,
                     torch.float64)
    r, miss, env_miss, rep = parity_fp64_vs_reference(*out, g)
    print(name, r)
    assert r["frac"] >= FP64_TOL_FRAC, (name, r, rep[:8])
    assert r["env_miss"] <= 1, (name, r)


def test_single_call_fp64_vs_reference_pooled(engines):
    """Pooled over all 14,080 fixture columns: >= 98.5 % inside the x10 bar."""
    tot = dict(nontie=0, tight=0, miss=0, env_miss=0, tie=0)
    for name in single_names():
        g = load(f"single_{name}.npz")
        out = run_single(engines(g["options"], 8, tags=fixture_tags(g)), g, torch.float64)
        r = parity_fp64_vs_reference(*out, g)[0]
        for k in tot:
            tot[k] += r[k]
    print("fp64 vs reference, pooled:", tot, tot["tight"] / tot["nontie"])
    assert tot["tight"] / tot["nontie"] >= FP64_POOLED_FRAC, tot
    assert tot["env_miss"] <= 2, tot


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", ["casenml", "combo_a", "snow"])
def test_trajectory_fp64_vs_reference(engines, name, variant):
    """fp64 engine along the reference trajectories at the x10 bar
    (golden_io.check_fp64_trajectory_step): the run/case.nml column inside
    rel 1e-3 at every saved step, snow by domain means within 1 %."""
    g = load(f"traj_{name}.npz")
    out = _trajectory(engines(g["options"], 8, variant=variant), g, torch.float64)
    for k, (st, isn, dg, _) in enumerate(out):
        step = min((k + 1) * int(g["keep_every"]) - 1, g["forcing"].shape[0] - 1)
        check_fp64_trajectory_step(name, step, st, isn, dg, g, k)


def test_config2_replicated_casenml_fp64(engines):
    """BASELINE config #2: 65,536 replicated run/case.nml columns, 4 soil / 0
    snow layers, fp64, one GPU.  The reference's 96-step case.nml column
    (traj_casenml column 0) is replicated 65,536 times and stepped through all
    96 steps: every replica stays bit-identical to the first (one launch, all
    1,024 waves), and the column meets the x10 trajectory bar against the
    reference at every saved step."""
    from noahmp_amd.engine import ColumnState
    g = load("traj_casenml.npz")
    n = 65536
    assert (g["isnows"][:, 0] == 0).all() and g["isnow0"][0] == 0  # 0 snow layers throughout
    rep = lambda a: np.ascontiguousarray(np.repeat(a[..., :1], n, axis=-1))
    cols = cases.ColumnSet(rep(g["static_f"]), rep(g["static_i"]), rep(g["state0"]),
                           rep(g["isnow0"]), *([None] * 7))
    eng = engines(g["options"], 8)
    cs = ColumnState.from_host(cols, DEV, torch.float64)
    F = torch.as_tensor(rep(g["forcing"]), device=DEV).to(torch.float64).contiguous()
    diag = torch.zeros((L.NDIAG_FULL, n), dtype=torch.float64, device=DEV)
    dt, ke = float(g["dt"]), int(g["keep_every"])
    k = 0
    for s in range(F.shape[0]):
        eng.step(cs, F[s], g["zsoil"], dt, float(g["julian0"]) + s * dt / 86400.0,
                 int(g["yearlen"]), diag, L.DIAG_FULL_LEVEL)
        if (s + 1) % ke == 0 or s == F.shape[0] - 1:
            torch.cuda.synchronize()
            bits = lambda t: t.view(torch.int64)
            assert torch.equal(bits(cs.state), bits(cs.state[:, :1]).expand(-1, n)), s
            assert torch.equal(bits(diag), bits(diag[:, :1]).expand(-1, n)), s
            assert bool((cs.isnow == 0).all()) and bool((cs.status == cs.status[0]).all())
            sub = lambda t: np.concatenate([t[:, :1].cpu().numpy(), g["states"][k][:, 1:]], 1)
            st = sub(cs.state)
            dg = np.concatenate([diag[:, :1].cpu().numpy(), g["diags"][k][:, 1:]], 1)
            isn = np.concatenate([cs.isnow[:1].cpu().numpy(), g["isnows"][k][1:]])
            check_fp64_trajectory_step("casenml", s, st, isn, dg, g, k)
            k += 1
    assert k == g["states"].shape[0]


def test_single_call_fast_math(engines):
    """ocml fp32 math (opt-in production mode): looser bar, same structure."""
    for name in ("casenml_mixed", "casenml_conus"):
        g = load(f"single_{name}.npz")
        r, msg = parity_vs_reference(*run_single(engines(g["options"], 4, "fast"), g), g,
                                     tol_frac=0.85, loose_frac=0.98, tie_frac=0.03)
        print("fast", name, r)
        assert not msg, f"fast {name}: {msg}"


def _trajectory(eng, g, dtype=torch.float32):
    from noahmp_amd.engine import ColumnState
    cols = cases.ColumnSet(g["static_f"], g["static_i"], g["state0"], g["isnow0"], *([None] * 7))
    cs = ColumnState.from_host(cols, DEV, dtype)
    F = torch.as_tensor(g["forcing"], device=DEV).to(dtype).contiguous()
    diag = torch.zeros((L.NDIAG_FULL, cs.ncol), dtype=dtype, device=DEV)
    dt, ke = float(g["dt"]), int(g["keep_every"])
    out = []
    for s in range(F.shape[0]):
        jul = float(g["julian0"]) + s * dt / 86400.0
        eng.step(cs, F[s], g["zsoil"], dt, jul, int(g["yearlen"]), diag, L.DIAG_FULL_LEVEL)
        if (s + 1) % ke == 0 or s == F.shape[0] - 1:
            out.append((cs.state.cpu().numpy(), cs.isnow.cpu().numpy(), diag.cpu().numpy(),
                        cs.status.cpu().numpy()))
    return out


@pytest.mark.parametrize("variant", VARIANTS32)
def test_trajectory_casenml(engines, variant):
    """96 steps of the case.nml column + 31 mixed columns vs the reference run."""
    g = load("traj_casenml.npz")
    out = _trajectory(engines(g["options"], variant=variant), g)
    for k in range(0, len(out), 8):
        st, isn = out[k][0], out[k][1]
        exp = g["states"][k]
        snowfree = (g["isnows"][:k + 1] == 0).all(0) & (g["isnow0"] == 0)
        ok = close(st[:, snowfree], exp[:, snowfree], 1e-4, 1e-4).all(0)
        assert ok.mean() >= 0.9, (k, column_mismatch(st[:, snowfree], exp[:, snowfree], 1e-4,
                                                      1e-4, STATE_NAMES)[1][:8])
        assert (isn == g["isnows"][k]).mean() >= 0.95, k
    # column 0 is the run/case.nml column itself
    np.testing.assert_allclose(out[-1][0][:, 0], g["states"][-1][:, 0], rtol=1e-4, atol=1e-4)
    # with glibc-exact math the whole 96-step run is bit-identical to the reference
    for k, (st, isn, dg, status) in enumerate(out):
        ex = bit_equal(st, g["states"][k]).all(0) & bit_equal(dg, g["diags"][k]).all(0)
        assert ex.all(), (k, ex.mean())


@pytest.mark.parametrize("variant", VARIANTS32)
def test_trajectory_snow_distribution(engines, variant):
    """480 snow steps: domain means (SWE, depth, cover) within 1 %, as SURVEY 8c asks."""
    g = load("traj_snow.npz")
    out = _trajectory(engines(g["options"], variant=variant), g)
    for k, (st, isn, dg, _) in enumerate(out):
        exp = g["states"][k]
        for f in ("SNEQV", "SNOWH"):
            a, b = st[L.si(f)].mean(), exp[L.si(f)].mean()
            assert abs(a - b) <= 0.01 * abs(b) + 1e-3, (k, f, a, b)
        assert abs((isn < 0).mean() - (g["isnows"][k] < 0).mean()) <= 0.01 + 1.0 / isn.size
        stc = L.s("STC")
        assert np.nanmean(np.abs(st[stc][3:] - exp[stc][3:])) < 0.5
    for k, (st, isn, dg, status) in enumerate(out):
        ex = bit_equal(st, g["states"][k]).all(0) & (isn == g["isnows"][k]) & \
            bit_equal(dg, g["diags"][k]).all(0)
        assert ex.all(), (k, ex.mean())


@pytest.mark.parametrize("variant", VARIANTS32)
def test_trajectory_option_combo(engines, variant):
    """48 steps under combo_a (dynamic vegetation + carbon, Jarvis canopy
    resistance, Chen97 surface layer, ... -- tests/golden/make_golden.py):
    bit-exact to the reference at every step."""
    g = load("traj_combo_a.npz")
    out = _trajectory(engines(g["options"], variant=variant), g)
    for k, (st, isn, dg, status) in enumerate(out):
        ex = bit_equal(st, g["states"][k]).all(0) & (isn == g["isnows"][k]) & \
            bit_equal(dg, g["diags"][k]).all(0) & (as_ref_status(status) == g["statuses"][k])
        assert ex.all(), (k, ex.mean())


def test_run_equals_repeated_step(engines):
    """nmp_run over a forcing cycle == the same steps issued one by one (bitwise)."""
    from noahmp_amd.engine import ColumnState
    g = load("traj_casenml.npz")
    eng = engines(g["options"])
    cols = cases.ColumnSet(g["static_f"], g["static_i"], g["state0"], g["isnow0"], *([None] * 7))
    F = torch.as_tensor(g["forcing"][:8], device=DEV).contiguous()
    dt = float(g["dt"])
    a = ColumnState.from_host(cols, DEV)
    b = ColumnState.from_host(cols, DEV)
    da = torch.zeros((L.NDIAG_OUT, a.ncol), device=DEV)
    db = torch.zeros_like(da)
    eng.run(a, F, g["zsoil"], dt, float(g["julian0"]), int(g["yearlen"]), 12, da,
            L.DIAG_OUT_LEVEL)
    for s in range(12):
        eng.step(b, F[s % 8], g["zsoil"], dt, float(g["julian0"]) + s * dt / 86400.0,
                 int(g["yearlen"]), db if s == 11 else None,
                 L.DIAG_OUT_LEVEL if s == 11 else L.DIAG_NONE)
    torch.cuda.synchronize()
    assert torch.equal(a.state, b.state) and torch.equal(a.isnow, b.isnow)
    assert torch.equal(da, db) and torch.equal(a.status, b.status)


def test_run_out_ring_equals_repeated_step(engines):
    """nmp_run_out == 12 nmp_step calls, bitwise: state, ISNOW, status, and each
    output step's diagnostics in its ring slot (out_every 3, 3 slots: the 4th
    output wraps onto slot 0); 200,003 columns = a ragged last block."""
    from noahmp_amd.engine import ColumnState
    from noahmp_amd.params import Params
    n, nsteps, every, slots = 200_003, 12, 3, 3
    opts = L.CASE_NML_OPTIONS
    eng = engines([opts[k] for k in L.OPTION_NAMES])
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=5, julian=100.0)
    F = torch.stack([torch.as_tensor(cases.forcing_step(cols, 100.0 + s * 1800.0 / 86400.0, 365,
                                                        s, seed=5)) for s in range(5)]).to(DEV)
    a = ColumnState.from_host(cols, DEV)
    b = ColumnState.from_host(cols, DEV)
    ring = torch.full((slots, L.NDIAG_OUT, n), float("nan"), device=DEV)
    eng.run(a, F, cases.CASE_NML_ZSOIL, 1800.0, 100.0, 365, nsteps, ring, L.DIAG_OUT_LEVEL,
            out_every=every)
    expect = {}
    d = torch.zeros((L.NDIAG_OUT, n), device=DEV)
    for s in range(nsteps):
        out = (s + 1) % every == 0
        jul = float(np.float32(100.0) + np.float32(s) * np.float32(1800.0) / np.float32(86400.0))
        eng.step(b, F[s % 5], cases.CASE_NML_ZSOIL, 1800.0, jul, 365, d if out else None,
                 L.DIAG_OUT_LEVEL if out else L.DIAG_NONE)
        if out:
            expect[((s + 1) // every - 1) % slots] = d.clone()
    torch.cuda.synchronize()
    bits = lambda t: t.view(torch.int32)  # NaN-safe bitwise comparison
    assert torch.equal(bits(a.state), bits(b.state)) and torch.equal(a.isnow, b.isnow)
    assert torch.equal(a.status, b.status)
    for k in range(slots):
        assert torch.equal(bits(ring[k]), bits(expect[k])), k


@pytest.mark.parametrize("nshards", [2, 3])
def test_stream_shards_equal_single_launch(engines, nshards):
    """Column ranges on their own streams (engine.StreamShards, the bench and
    driver default) == one launch per step, bitwise, over 6 steps with
    diagnostics on alternate steps; 200,003 columns = ragged ranges."""
    from noahmp_amd.engine import ColumnState, StreamShards
    from noahmp_amd.params import Params
    n = 200_003
    eng = engines([L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES])
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=6, julian=200.0)
    F = [torch.as_tensor(cases.forcing_step(cols, 200.0 + s / 48.0, 365, s, seed=6), device=DEV)
         for s in range(6)]
    a = ColumnState.from_host(cols, DEV)
    b = ColumnState.from_host(cols, DEV)
    sh = StreamShards(eng, a, nshards)
    da = [torch.zeros((L.NDIAG_OUT, n), device=DEV) for _ in range(3)]
    db = [torch.zeros((L.NDIAG_OUT, n), device=DEV) for _ in range(3)]
    for s in range(6):
        out = s % 2 == 1
        lvl = L.DIAG_OUT_LEVEL if out else L.DIAG_NONE
        sh.step(F[s], cases.CASE_NML_ZSOIL, 1800.0, 200.0 + s / 48.0, 365,
                da[s // 2] if out else None, lvl)
        eng.step(b, F[s], cases.CASE_NML_ZSOIL, 1800.0, 200.0 + s / 48.0, 365,
                 db[s // 2] if out else None, lvl)
    sh.join()
    torch.cuda.synchronize()
    bits = lambda t: t.view(torch.int32)
    assert torch.equal(bits(a.state), bits(b.state)) and torch.equal(a.isnow, b.isnow)
    assert torch.equal(a.status, b.status)
    for x, y in zip(da, db):
        assert torch.equal(bits(x), bits(y))


@pytest.mark.parametrize("tile,every", [(1024, 1), (4096, 2)])
def test_rebinned_steps_equal_plain_steps(engines, tile, every):
    """Column re-binning (StreamShards rebin_tile / nmp_step_binned + nmp_rebin)
    only changes which lane steps which column: state, ISNOW, status and every
    output step's diagnostics are bit-identical to plain launches over 6 steps;
    200,003 columns = ragged ranges and a ragged last tile."""
    from noahmp_amd.engine import ColumnState, StreamShards
    from noahmp_amd.params import Params
    n = 200_003
    eng = engines([L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES])
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=7, julian=200.0)
    F = [torch.as_tensor(cases.forcing_step(cols, 200.0 + s / 48.0, 365, s, seed=7), device=DEV)
         for s in range(6)]
    a = ColumnState.from_host(cols, DEV)
    b = ColumnState.from_host(cols, DEV)
    sa = StreamShards(eng, a, 2, rebin_tile=tile, rebin_every=every)
    sb = StreamShards(eng, b, 2)
    da = [torch.zeros((L.NDIAG_OUT, n), device=DEV) for _ in range(3)]
    db = [torch.zeros((L.NDIAG_OUT, n), device=DEV) for _ in range(3)]
    for s in range(6):
        out = s % 2 == 1
        lvl = L.DIAG_OUT_LEVEL if out else L.DIAG_NONE
        for sh, d in ((sa, da), (sb, db)):
            sh.step(F[s], cases.CASE_NML_ZSOIL, 1800.0, 200.0 + s / 48.0, 365,
                    d[s // 2] if out else None, lvl)
    sa.join()
    sb.join()
    torch.cuda.synchronize()
    bits = lambda t: t.view(torch.int32)
    assert torch.equal(bits(a.state), bits(b.state)) and torch.equal(a.isnow, b.isnow)
    assert torch.equal(a.status, b.status)
    for x, y in zip(da, db):
        assert torch.equal(bits(x), bits(y))
    # the order really was permuted: each range's order is a permutation of its columns
    # and not the identity
    for lo, hi in sa.ranges:
        o = sa.order[lo:hi].cpu().numpy()
        assert np.array_equal(np.sort(o), np.arange(hi - lo))
        assert (o != np.arange(hi - lo)).any()


def test_step_binned_order_check(engines, monkeypatch):
    """nmp_step_binned trusts `order` (noahmp_engine.h precondition);
    NMP_CHECK_ORDER=1 makes Engine.step refuse a non-permutation before any
    launch, and pass a real one."""
    from noahmp_amd.engine import ColumnState
    from noahmp_amd.params import Params
    n = 1000
    eng = engines([L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES])
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=3, julian=200.0)
    F = torch.as_tensor(cases.forcing_step(cols, 200.0, 365, 0, seed=3), device=DEV)
    cs = ColumnState.from_host(cols, DEV)
    before = cs.state.clone()
    monkeypatch.setenv("NMP_CHECK_ORDER", "1")
    bad = torch.arange(n, dtype=torch.int32, device=DEV)
    bad[5] = 4  # duplicate
    for o in (bad, torch.full((n,), n, dtype=torch.int32, device=DEV)):
        with pytest.raises(ValueError, match="not a permutation"):
            eng.step(cs, F, cases.CASE_NML_ZSOIL, 1800.0, 200.0, 365, order=o)
    torch.cuda.synchronize()
    assert torch.equal(cs.state.view(torch.int32), before.view(torch.int32))
    good = torch.flip(torch.arange(n, dtype=torch.int32, device=DEV), (0,))
    eng.step(cs, F, cases.CASE_NML_ZSOIL, 1800.0, 200.0, 365, order=good)
    torch.cuda.synchronize()


@pytest.mark.parametrize("opt_veg,precision", [(1, 4), (2, 4), (1, 8), (2, 8)])
def test_option_set_kernels_equal_generic(opt_veg, precision):
    """The compiled option-set kernels (case.nml options = set 1, + opt_veg 2
    = set 2) == the run-time-options kernel (set 0), bitwise, over 4 steps of
    120,001 mixed columns with output on alternate steps -- ragged, every
    vegetation/soil type, snow, water and ice columns."""
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.params import Params
    n = 120_001
    opts = dict(L.CASE_NML_OPTIONS, opt_veg=opt_veg)
    tab = Params.builtin()
    a_eng = Engine(tab, opts, device=0, precision=precision)
    b_eng = Engine(tab, opts, device=0, precision=precision)
    try:
        assert a_eng.option_set() == opt_veg  # kOptionSet[1] / [2]
        assert b_eng.option_set(0) == 0 and b_eng.option_set() == 0
        dtype = torch.float32 if precision == 4 else torch.float64
        cols = cases.make_columns(n, "mixed", tab.as_dict(), seed=11, julian=170.0)
        F = [torch.as_tensor(cases.forcing_step(cols, 170.0 + s / 48.0, 365, s, seed=11),
                             device=DEV).to(dtype) for s in range(4)]
        a = ColumnState.from_host(cols, DEV, dtype)
        b = ColumnState.from_host(cols, DEV, dtype)
        for s in range(4):
            lvl = L.DIAG_FULL_LEVEL if s % 2 else L.DIAG_NONE
            da = torch.zeros((L.NDIAG_FULL, n), dtype=dtype, device=DEV) if s % 2 else None
            db = torch.zeros((L.NDIAG_FULL, n), dtype=dtype, device=DEV) if s % 2 else None
            for eng, cs, d in ((a_eng, a, da), (b_eng, b, db)):
                eng.step(cs, F[s], cases.CASE_NML_ZSOIL, 1800.0, 170.0 + s / 48.0, 365, d, lvl)
            torch.cuda.synchronize()
            if d is not None:
                assert torch.equal(da.view(torch.int8), db.view(torch.int8)), s
        assert torch.equal(a.state.view(torch.int8), b.state.view(torch.int8))
        assert torch.equal(a.isnow, b.isnow) and torch.equal(a.status, b.status)
        # set 1 is picked back when asked; another option combination has no set
        assert b_eng.option_set(1) == opt_veg
    finally:
        a_eng.close()
        b_eng.close()
    c_eng = Engine(tab, dict(opts, opt_run=2), device=0, precision=precision)
    assert c_eng.option_set() == 0
    c_eng.close()


def _combo_options(name):
    return [int(x) for x in load(f"single_combo_{name}.npz")["options"]]


@pytest.mark.parametrize("precision", [4, 8])
@pytest.mark.parametrize("optset", ["set1", "set2", "set0_casenml", "set0_combo_a",
                                    "set0_combo_b", "set0_combo_c"])
def test_full_and_small_kernels_equal(optset, precision):
    """The full-occupancy kernel (what every production-size launch runs) ==
    the half-occupancy kernel (what the fixture sizes select), bitwise, for
    every compiled option set and for the run-time-options kernel under
    case.nml and under the hand-picked option combinations (which together set
    every option to a non-default value): 4 steps of 200,003 mixed columns
    (ragged), full diagnostics on alternate steps.  Round 3's ballot build got
    91,067 columns wrong in exactly this comparison while every fixture test
    (half occupancy) passed."""
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.params import Params
    n = 200_003
    if optset.startswith("set0_combo"):
        opts = dict(zip(L.OPTION_NAMES, _combo_options(optset[len("set0_combo_"):])))
    else:
        opts = dict(L.CASE_NML_OPTIONS, opt_veg=2 if optset == "set2" else 1)
    tab = Params.builtin()
    engs = [Engine(tab, opts, device=0, precision=precision) for _ in range(2)]
    try:
        if optset.startswith("set0"):
            for e in engs:
                e.option_set(0)
        assert engs[0].option_set() == {"set1": 1, "set2": 2}.get(optset, 0)
        assert engs[0].launch_variant("small") == "small"
        assert engs[1].launch_variant("full") == "full"
        dtype = torch.float32 if precision == 4 else torch.float64
        cols = cases.make_columns(n, "mixed", tab.as_dict(), seed=13, julian=60.0)
        F = [torch.as_tensor(cases.forcing_step(cols, 60.0 + s / 48.0, 365, s, seed=13),
                             device=DEV).to(dtype) for s in range(4)]
        cs = [ColumnState.from_host(cols, DEV, dtype) for _ in range(2)]
        nbytes = torch.int8
        for s in range(4):
            lvl = L.DIAG_FULL_LEVEL if s % 2 else L.DIAG_NONE
            d = [torch.zeros((L.NDIAG_FULL, n), dtype=dtype, device=DEV) if s % 2 else None
                 for _ in range(2)]
            for e, c, dd in zip(engs, cs, d):
                e.step(c, F[s], cases.CASE_NML_ZSOIL, 1800.0, 60.0 + s / 48.0, 365, dd, lvl)
            torch.cuda.synchronize()
            if s % 2:
                diff = (d[0].view(nbytes) != d[1].view(nbytes)).any(0).sum().item()
                assert diff == 0, f"step {s}: {diff} columns' diagnostics differ"
        bad = (cs[0].state.view(nbytes) != cs[1].state.view(nbytes)).any(0)
        assert not bool(bad.any()), f"{int(bad.sum())} columns' state differ"
        assert torch.equal(cs[0].isnow, cs[1].isnow) and torch.equal(cs[0].status, cs[1].status)
    finally:
        for e in engs:
            e.close()


def test_launch_variant_auto_picks_by_size(engines):
    """auto: the half-occupancy kernel for launches within its wave slots, the
    full one above; small/full stick for every size; bad requests are refused."""
    from noahmp_amd import lib as _lib
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    e = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0)
    try:
        assert e.launch_variant() == "auto"
        assert e.launch_variant("full") == "full" and e.launch_variant() == "full"
        assert e.launch_variant("small") == "small"
        assert e.launch_variant("auto") == "auto"
        with pytest.raises(_lib.NmpError):
            e.launch_variant(3)
        assert e.launch_variant() == "auto"
    finally:
        e.close()


@pytest.mark.parametrize("cpw", [8, 24, 40, 64])
def test_cols_per_wave_bit_identical(engines, cpw):
    """Columns per wave (nmp_set_cols_per_wave) only changes the lane -> column
    map: every cpw gives the reference's bits on the mixed fixture, with a
    ragged column count (2,047) so the last wave and block are partial."""
    from noahmp_amd.params import Params
    g = load("single_casenml_mixed.npz")
    n = 2047
    sub = {k: (v[..., :n] if isinstance(v, np.ndarray) and v.ndim >= 1 and
               v.shape[-1] == g["isnow0"].shape[0] else v) for k, v in g.items()}
    from noahmp_amd.engine import Engine
    eng = Engine(Params.builtin(), dict(zip(L.OPTION_NAMES, g["options"].tolist())), device=0)
    eng.set_cols_per_wave(cpw)
    st, isn, dg, status = run_single(eng, sub)
    eng.close()
    ok = bit_equal(st, sub["state1"]).all(0) & bit_equal(dg, sub["diag"]).all(0) & \
        (isn == sub["isnow1"])
    assert ok.all(), (~ok).sum()


def test_small_column_set_cols_per_wave_fp64(engines):
    """A small fp64 set (65,536 columns) at 32 columns per wave gives the same
    bits as full waves."""
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.params import Params
    n = 65536
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=9, julian=120.0)
    f = torch.as_tensor(cases.forcing_step(cols, 120.0, 366, 0, seed=9), device=DEV).double()
    out = []
    for cpw in (32, 64):
        eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=8)
        eng.set_cols_per_wave(cpw)
        cs = ColumnState.from_host(cols, DEV, torch.float64)
        d = torch.zeros((L.NDIAG_OUT, n), dtype=torch.float64, device=DEV)
        eng.step(cs, f, cases.CASE_NML_ZSOIL, 1800.0, 120.0, 366, d, L.DIAG_OUT_LEVEL)
        torch.cuda.synchronize()
        out.append((cs.state.view(torch.int64).clone(), d.view(torch.int64).clone()))
        eng.close()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def test_cost_key_is_the_reference_trip_count(engines, oracle_port):
    """The re-binning key the kernel records (nmp_step_binned cost) is the
    vege_flux Newton trip count, equal to the oracle's count for every column
    of the mixed fixture (0 where no canopy flux is computed)."""
    from noahmp_amd.engine import ColumnState
    g = load("single_casenml_mixed.npz")
    eng = engines(g["options"])
    cols = cases.ColumnSet(g["static_f"], g["static_i"], g["state0"], g["isnow0"], *([None] * 7))
    cs = ColumnState.from_host(cols, DEV)
    n = cs.ncol
    cost = torch.full((n,), 255, dtype=torch.uint8, device=DEV)
    order = torch.as_tensor(np.random.default_rng(0).permutation(n).astype(np.int32), device=DEV)
    f = torch.as_tensor(g["forcing"], device=DEV).contiguous()
    eng.step(cs, f, g["zsoil"], float(g["dt"]), float(g["julian"]), int(g["yearlen"]),
             order=order, cost=cost)
    torch.cuda.synchronize()
    *_, it = oracle_port.step_stats(load_params(), tuple(g["options"]), g["zsoil"], float(g["dt"]),
                                    int(g["yearlen"]), float(g["julian"]), g["state0"],
                                    g["isnow0"], g["static_f"], g["static_i"], g["forcing"])
    assert np.array_equal(cost.cpu().numpy(), it[:, 0].astype(np.uint8))
    assert bit_equal(cs.state.cpu().numpy(), g["state1"]).all()  # a random order, same bits


_SINGLE_FIXTURES = ["single_" + n for n in single_names()]


@pytest.mark.parametrize("precision", [4, 8])
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", _SINGLE_FIXTURES)
def test_diag_levels_consistent(engines, name, variant, precision):
    """DIAG_OUT fields are the DIAG_FULL values (T2M = the fveg blend of
    T2MV/T2MB), and the state is the same bits at every diagnostics level --
    with no diagnostics the kernel skips the 2-m chain (MOZ2 -> FH2 -> CHV2,
    CHB2 -> T2M, Q2), which nothing else reads -- for every single-call
    fixture (every option value and table pair), on both occupancy kernels,
    in fp32 and fp64."""
    from noahmp_amd.engine import ColumnState
    g = load(name + ".npz")
    eng = engines(g["options"], precision=precision, variant=variant)
    dtype = torch.float32 if precision == 4 else torch.float64
    cols = cases.ColumnSet(g["static_f"], g["static_i"], g["state0"], g["isnow0"], *([None] * 7))
    f = torch.as_tensor(g["forcing"], device=DEV).to(dtype).contiguous()
    outs = {}
    for lvl, nd in ((L.DIAG_FULL_LEVEL, L.NDIAG_FULL), (L.DIAG_OUT_LEVEL, L.NDIAG_OUT),
                    (L.DIAG_NONE, 0)):
        cs = ColumnState.from_host(cols, DEV, dtype)
        d = torch.zeros((max(nd, 1), cs.ncol), dtype=dtype, device=DEV) if nd else None
        eng.step(cs, f, g["zsoil"], float(g["dt"]), float(g["julian"]), int(g["yearlen"]), d, lvl)
        torch.cuda.synchronize()
        outs[lvl] = (cs.state.cpu().numpy(), None if d is None else d.cpu().numpy())
    full, out = outs[L.DIAG_FULL_LEVEL][1], outs[L.DIAG_OUT_LEVEL][1]
    for i, n in enumerate(L.DIAG_OUT):
        if n != "T2M":
            np.testing.assert_array_equal(out[i], full[L.DIAG_FULL.index(n)], err_msg=n)
    if name == "single_casenml_conus" and precision == 4:
        fveg = full[L.DIAG_FULL.index("FVEG")]
        t2m = out[L.DIAG_OUT.index("T2M")]
        veg = g["static_i"][L.STATIC_I.index("IST")] == 1
        blend = fveg * full[L.DIAG_FULL.index("T2MV")] + (1 - fveg) * full[L.DIAG_FULL.index("T2MB")]
        np.testing.assert_allclose(t2m[veg & (fveg > 0)], blend[veg & (fveg > 0)], rtol=1e-5)
    for lvl in (L.DIAG_OUT_LEVEL, L.DIAG_NONE):
        assert bit_equal(outs[lvl][0], outs[L.DIAG_FULL_LEVEL][0]).all(), lvl


def test_ragged_and_empty(engines):
    """ncol = 0, 1 and a non-multiple of the block size; ld > ncol."""
    from noahmp_amd import lib as _lib
    from noahmp_amd.engine import ColumnState
    import ctypes as C
    g = load("single_casenml_mixed.npz")
    eng = engines(g["options"])
    for n in (1, 63, 257):
        sub = {k: (v[..., :n] if isinstance(v, np.ndarray) and v.ndim >= 1 and
                   v.shape[-1] == g["isnow0"].shape[0] else v) for k, v in g.items()}
        r, msg = parity_vs_reference(*run_single(eng, sub), sub)
        assert not msg, f"n={n}: {msg}"
    # empty launch is a no-op
    cols = cases.ColumnSet(g["static_f"][:, :0], g["static_i"][:, :0], g["state0"][:, :0],
                           g["isnow0"][:0], *([None] * 7))
    cs = ColumnState.from_host(cols, DEV)
    eng.step(cs, torch.zeros((L.NFORCING, 0), device=DEV), g["zsoil"], 1800.0, 1.0, 366)
    # ld > ncol: operate on the first 100 of 128 columns of padded buffers
    n, ld = 100, 128
    pad = lambda a, dt: torch.as_tensor(np.pad(a[..., :n], [(0, 0)] * (a.ndim - 1) + [(0, ld - n)]),
                                        device=DEV).to(dt).contiguous()
    st = pad(g["state0"], torch.float32)
    isn = pad(g["isnow0"], torch.int32)
    sf = pad(g["static_f"], torch.float32)
    si = pad(g["static_i"], torch.int32)
    fc = pad(g["forcing"], torch.float32)
    status = torch.zeros(ld, dtype=torch.int32, device=DEV)
    zs = (C.c_float * 4)(*g["zsoil"].tolist())
    _lib.check(eng._lib.nmp_step(eng._h, n, ld, zs, float(g["dt"]), float(g["julian"]),
                                 int(g["yearlen"]), st.data_ptr(), isn.data_ptr(), sf.data_ptr(),
                                 si.data_ptr(), fc.data_ptr(), None, 0, status.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    got = st.cpu().numpy()[:, :n]
    bad, rep = column_mismatch(got, g["state1"][:, :n], 1e-5, 1e-4, STATE_NAMES)
    assert bad.sum() <= 3, rep
    assert (st.cpu().numpy()[:, n:] == 0).all(), "wrote past ncol"


@pytest.mark.parametrize("name", ["casenml_mixed", "casenml_conus", "veg2", "fatal"])
def test_sflx_columns_reference_calling_sequence(engines, name):
    """nmp_sflx_columns: the 131 noahmp_sflx arguments per column (host records,
    include/noahmp_engine.h nmp_sflx_args) give the reference's results bit for
    bit, exactly as the SoA nmp_step path does."""
    g = load(f"single_{name}.npz")
    eng = engines(g["options"], tags=fixture_tags(g))
    r = L.sflx_records(g["state0"], g["isnow0"], g["static_f"], g["static_i"], g["forcing"],
                       g["zsoil"], g["dt"], g["julian"], g["yearlen"])
    eng.sflx_columns(r)
    st, isn, dg, status = L.soa_from_records(r)
    exact = bit_equal(st, g["state1"]).all(0) & bit_equal(dg, g["diag"]).all(0) & \
        (isn == g["isnow1"]) & (as_ref_status(status) == g["status"])
    assert exact.all(), f"{name}: {(~exact).sum()} columns differ"
    one = L.sflx_records(g["state0"][:, :1], g["isnow0"][:1], g["static_f"][:, :1],
                         g["static_i"][:, :1], g["forcing"][:, :1], g["zsoil"], g["dt"],
                         g["julian"], g["yearlen"])
    import ctypes as C
    assert eng._lib.nmp_sflx_column(eng._h, C.c_void_p(one.ctypes.data)) == 0
    assert bit_equal(L.soa_from_records(one)[0], g["state1"][:, :1]).all()


def test_sflx_columns_rejects_what_the_kernel_cannot_honour(engines):
    """Launch-wide arguments must agree across records (NMP_E_ARG otherwise)."""
    from noahmp_amd import lib as _lib
    g = load("single_casenml_mixed.npz")
    eng = engines(g["options"])
    ix = np.nonzero(g["isnow0"] < 0)[0][:8]  # snow-covered columns
    mk = lambda: L.sflx_records(g["state0"][:, ix], g["isnow0"][ix], g["static_f"][:, ix],
                                g["static_i"][:, ix], g["forcing"][:, ix], g["zsoil"], g["dt"],
                                g["julian"], g["yearlen"])
    r = mk()
    r["dt"][3] += 1.0
    with pytest.raises(_lib.NmpError):
        eng.sflx_columns(r)
    r = mk()
    r["nsoil"][0] = 5
    with pytest.raises(_lib.NmpError):
        eng.sflx_columns(r)
    assert eng.sflx_columns(mk()) is not None


def test_column_stride_limit_is_rejected(engines):
    """The kernels form a column's byte offset from each field's base in 32
    bits (sflx_kernel.hip col_at), so the host refuses a stride ld >= 2^29
    (engine.hip kMaxColumns) with NMP_E_ARG before any launch; 2^29 - 1 is
    only limited by the arrays the caller passes (not exercised: 2^29 columns
    of state are 120 GB)."""
    import ctypes as C
    from noahmp_amd import lib as _lib
    from noahmp_amd.engine import ColumnState
    from noahmp_amd.params import Params
    eng = engines([L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES])
    cols = cases.make_columns(256, "mixed", Params.builtin().as_dict(), seed=3, julian=180.0)
    cs = ColumnState.from_host(cols, DEV)
    f = torch.as_tensor(cases.forcing_step(cols, 180.0, 366, 0, seed=3), device=DEV)
    before = cs.state.clone()
    zs = (C.c_float * 4)(*[float(z) for z in cases.CASE_NML_ZSOIL])
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    s = C.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    for ld in (1 << 29, (1 << 31) + 256):
        rc = eng._lib.nmp_step(eng._h, 256, ld, zs, 1800.0, 180.0, 366, p(cs.state), p(cs.isnow),
                               p(cs.static_f), p(cs.static_i), p(f), None, L.DIAG_NONE,
                               p(cs.status), s)
        assert rc == -1, (ld, rc)  # NMP_E_ARG
    torch.cuda.synchronize()
    assert torch.equal(cs.state, before)


def test_julian_outside_the_year_is_rejected(engines):
    """The calendar position must be a day of the year, 0 <= julian <=
    yearlen (the reference's phenology indexes its 12-month LAI/SAI tables
    with it and reads out of bounds past the year's end): nmp_step, nmp_run
    (every step's julian0 + s*dt/86400) and nmp_sflx_columns return NMP_E_ARG,
    and the state is left untouched."""
    from noahmp_amd import lib as _lib
    from noahmp_amd.engine import ColumnState
    from noahmp_amd.params import Params
    eng = engines([L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES])
    cols = cases.make_columns(256, "mixed", Params.builtin().as_dict(), seed=3, julian=180.0)
    cs = ColumnState.from_host(cols, DEV)
    f = torch.as_tensor(cases.forcing_step(cols, 180.0, 366, 0, seed=3), device=DEV)
    before = cs.state.clone()
    for jul in (366.5, -0.25, float("nan")):
        with pytest.raises(_lib.NmpError):
            eng.step(cs, f, cases.CASE_NML_ZSOIL, 1800.0, jul, 366)
    # a run whose last step would pass the year's end (365.9 + 4 x 1 h)
    F = f.unsqueeze(0).repeat(4, 1, 1)
    with pytest.raises(_lib.NmpError):
        eng.run(cs, F, cases.CASE_NML_ZSOIL, 3600.0, 365.9, 366, 4)
    torch.cuda.synchronize()
    assert torch.equal(cs.state, before)
    g = load("single_casenml_mixed.npz")
    r = L.sflx_records(g["state0"][:, :4], g["isnow0"][:4], g["static_f"][:, :4],
                       g["static_i"][:, :4], g["forcing"][:, :4], g["zsoil"], g["dt"],
                       np.float32(g["yearlen"]) + 1.0, g["yearlen"])
    with pytest.raises(_lib.NmpError):
        engines(g["options"]).sflx_columns(r)
    # the year's last instant itself is accepted
    eng.step(cs, f, cases.CASE_NML_ZSOIL, 1800.0, 366.0, 366)
    torch.cuda.synchronize()


def test_sflx_columns_caller_ficeold_vs_reference(engines):
    """nmp_sflx_columns takes FICEOLD as the record carries it (noahmp_sflx's
    intent(in) argument, func.f90:129): melting snow columns whose caller
    FICEOLD differs from the step-start ice fraction give the reference's bits
    (tests/golden/ficeold_snow.npz, made by the reference with that FICEOLD)."""
    g = load("ficeold_snow.npz")
    eng = engines(g["options"])
    r = L.sflx_records(g["state0"], g["isnow0"], g["static_f"], g["static_i"], g["forcing"],
                       g["zsoil"], g["dt"], g["julian"], g["yearlen"])
    r["ficeold"][:] = g["ficeold"].T
    eng.sflx_columns(r)
    st, isn, dg, status = L.soa_from_records(r)
    exact = bit_equal(st, g["state1"]).all(0) & bit_equal(dg, g["diag"]).all(0) & \
        (isn == g["isnow1"]) & (as_ref_status(status) == g["status"])
    _, rep_s = column_mismatch(st, g["state1"], 0, 0, STATE_NAMES)
    _, rep_d = column_mismatch(dg, g["diag"], 0, 0, L.DIAG_FULL)
    assert exact.all(), f"{(~exact).sum()} of {exact.size} columns differ: " + "; ".join(
        rep_s[:8] + rep_d[:8])


@pytest.mark.parametrize("kind,ncol,opt_veg,precision", [
    ("mixed", 1 << 20, 1, 4),          # config #3 as the bench runs it
    ("global", 1_036_800, 2, 4),       # config #5 grid + carbon, fp32
    ("global", 1_036_800, 2, 8),       # config #5 in fp64 (vs the fp64 restatement)
    ("casenml", 65536, 1, 8),          # config #2: replicated case.nml columns, fp64
    ("conus", 524_288, 1, 4),          # config #4: one of 8 shards of the CONUS-like grid
    ("conus", 4_194_304, 1, 4),        # config #4 whole: all 4,194,304 columns on one GPU
])
def test_full_size_sample_vs_oracle(engines, oracle_port, kind, ncol, opt_veg, precision):
    """BASELINE sizes: two steps of every column on the GPU, then a seeded
    sample of 2,048 columns re-run through the C restatement (JULIAN is a real
    argument of noahmp_sflx and of nmp_step, fp32 in every precision, so the
    oracle gets the same fp32 value; the restatement is bit-exact to the
    reference in fp32 on every fixture): bit-identical in fp32, |d| <= 1e-9
    (1 + |x|) in fp64.  Column independence makes the sample a full check of
    those columns at full launch size (grid, stream ranges, ragged tail)."""
    from noahmp_amd.engine import ColumnState, StreamShards
    from noahmp_amd.params import Params
    P = Params.builtin()
    opts = dict(L.CASE_NML_OPTIONS, opt_veg=opt_veg)
    eng = engines([opts[k] for k in L.OPTION_NAMES], precision)
    dtype = torch.float32 if precision == 4 else torch.float64
    cols = cases.make_columns(ncol, kind, P.as_dict(), seed=11, julian=150.0)
    dt, jul = 1800.0, [150.0, 150.0 + 1800.0 / 86400.0]
    F = [cases.forcing_step(cols, j, 366, s, seed=11) for s, j in enumerate(jul)]
    cs = ColumnState.from_host(cols, DEV, dtype)
    sh = StreamShards(eng, cs, 2)
    diag = torch.zeros((L.NDIAG_OUT, ncol), dtype=dtype, device=DEV)
    for s in range(2):
        sh.step(torch.as_tensor(F[s], device=DEV).to(dtype), cases.CASE_NML_ZSOIL, dt, jul[s], 366,
                diag if s == 1 else None, L.DIAG_OUT_LEVEL if s == 1 else L.DIAG_NONE)
    sh.join()
    torch.cuda.synchronize()
    idx = np.sort(np.random.default_rng(3).choice(ncol, 2048, replace=False))
    idx[-1] = ncol - 1  # the ragged tail's last column
    st, isn = cols.state[:, idx], cols.isnow[idx]
    for s in range(2):
        st, isn, dg, status = oracle_port.step(
            load_params(), tuple(opts[k] for k in L.OPTION_NAMES), cases.CASE_NML_ZSOIL, dt, 366,
            float(np.float32(jul[s])), st, isn, cols.static_f[:, idx], cols.static_i[:, idx], F[s][:, idx],
            precision=precision)
    got = cs.state.cpu().numpy()[:, idx]
    gd = diag.cpu().numpy()[:, idx]
    od = np.stack([dg[L.DIAG_FULL.index(n)] for n in L.DIAG_OUT if n != "T2M"])
    gd = np.stack([gd[i] for i, n in enumerate(L.DIAG_OUT) if n != "T2M"])
    assert np.array_equal(cs.isnow.cpu().numpy()[idx], isn)
    if precision == 4:
        ok = bit_equal(got, st).all(0) & bit_equal(gd, od).all(0)
        assert ok.all(), f"{(~ok).sum()} of {idx.size} sampled columns differ"
    else:
        ok = close(got, st, 1e-9, 1e-9).all(0) & close(gd, od, 1e-9, 1e-9).all(0)
        assert ok.mean() >= 0.99, column_mismatch(got, st, 1e-9, 1e-9, STATE_NAMES)[1][:8]


@pytest.mark.parametrize("rank", [0, 3])
def test_config5_shard_bench_pipeline_vs_oracle(engines, oracle_port, rank):
    """Config #5 as each of the 8 GPUs holds it: the
    129,600-column shard `bench.py --kind global --ncol 129600 --precision 8
    --opt-veg 2 --dt 3600 --out-every 1 --forcing device` steps on rank R
    (seed 1000 + R, global columns R x 129,600 on), in the coherent order, two
    stream ranges, forcing generated on each range's stream before its launch,
    carbon on, the 16 output fluxes every step -- the bench's own pipeline,
    emulated on one GPU (`--emulate-rank`).  Rank 0 is the polar band (ice
    sheets), rank 3 the southern subtropics.  Three steps, then a seeded
    sample of 2,048 columns through the fp64 restatement with the device's
    forcing: |d| <= 1e-9 (1 + |x|) on >= 99 % of columns, state and fluxes."""
    from noahmp_amd.engine import ColumnState, StreamShards
    from noahmp_amd.order import coherent_order
    from noahmp_amd.params import Params
    P = Params.builtin("STAS", "USGS")
    opts = dict(L.CASE_NML_OPTIONS, opt_veg=2)
    eng = engines([opts[k] for k in L.OPTION_NAMES], 8)
    n, dt, yl, seed, nsteps = 129_600, 3600.0, 366, 1000 + rank, 3
    cols = cases.make_columns(n, "global", P.as_dict(), seed=seed, julian=180.0, first=rank * n)
    cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, "lon-snow-type",
                                    band_deg=4.0))
    cs = ColumnState.from_host(cols, DEV, torch.float64)
    sh = StreamShards(eng, cs, 2)
    clim = torch.as_tensor(cases.climate(cols), device=DEV).contiguous()
    F = torch.empty((2, L.NFORCING, n), dtype=torch.float64, device=DEV)
    diag = torch.zeros((L.NDIAG_OUT, n), dtype=torch.float64, device=DEV)
    jul = [(180.0 + k * dt / 86400.0) % yl for k in range(nsteps)]
    forc = []
    for k in range(nsteps):
        f = F[k % 2]
        pre = lambda st, rng, f=f, k=k: eng.forcing_synth(  # noqa: E731
            clim, jul[k], yl, seed, k, f, first_col=rank * n, stream=st, cols=rng)
        sh.step(f, cases.CASE_NML_ZSOIL, dt, jul[k], yl, diag, L.DIAG_OUT_LEVEL, pre=pre)
        sh.join()
        torch.cuda.synchronize()
        forc.append(f.cpu().numpy().copy())
    idx = np.sort(np.random.default_rng(7).choice(n, 2048, replace=False))
    idx[-1] = n - 1
    st, isn = cols.state[:, idx], cols.isnow[idx]
    for k in range(nsteps):
        st, isn, dg, _ = oracle_port.step(
            load_params(), tuple(opts[x] for x in L.OPTION_NAMES), cases.CASE_NML_ZSOIL, dt, yl,
            float(np.float32(jul[k])), st, isn, cols.static_f[:, idx], cols.static_i[:, idx],
            forc[k][:, idx], precision=8)
    got = cs.state.cpu().numpy()[:, idx]
    gd = diag.cpu().numpy()[:, idx]
    od = np.stack([dg[L.DIAG_FULL.index(m)] for m in L.DIAG_OUT if m != "T2M"])
    gd = np.stack([gd[i] for i, m in enumerate(L.DIAG_OUT) if m != "T2M"])
    assert np.isfinite(got[L.s("STC")]).all()
    ok = close(got, st, 1e-9, 1e-9).all(0) & close(gd, od, 1e-9, 1e-9).all(0) & \
        (cs.isnow.cpu().numpy()[idx] == isn)
    assert ok.mean() >= 0.99, column_mismatch(got, st, 1e-9, 1e-9, STATE_NAMES)[1][:8]


def test_bench_window_bit_exact_vs_oracle(engines, oracle_port):
    """The workload bench.py times, as the driver runs it (`--steps 20
    --warmup 5`): config #3's 1,048,576 mixed columns in the coherent order,
    two stream ranges, resident forcing slices, julian wrapped at the year,
    output every 6th step -- all 25 steps, then a seeded sample of 2,048
    columns (and the last one) through the C restatement with the same
    inputs: state, ISNOW and the last output step's fluxes bit for bit."""
    from noahmp_amd.engine import ColumnState, StreamShards
    from noahmp_amd.order import coherent_order
    from noahmp_amd.params import Params
    P = Params.builtin("STAS", "USGS")
    opts = [L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES]
    eng = engines(opts)
    n, dt, yl, seed, nsteps, every = 1 << 20, 1800.0, 366, 1000, 25, 6
    cols = cases.make_columns(n, "mixed", P.as_dict(), seed=seed, julian=180.0)
    cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, "lon-snow-type"))
    jul = [float(np.float32((180.0 + k * dt / 86400.0) % yl)) for k in range(nsteps)]
    F = [cases.forcing_step(cols, (180.0 + k * dt / 86400.0) % yl, yl, k, seed=seed)
         for k in range(nsteps)]
    cs = ColumnState.from_host(cols, DEV)
    sh = StreamShards(eng, cs, 2)
    diag = torch.zeros((L.NDIAG_OUT, n), device=DEV)
    last = None
    for k in range(nsteps):
        out = (k + 1) % every == 0
        last = k if out else last
        sh.step(torch.as_tensor(F[k], device=DEV), cases.CASE_NML_ZSOIL, dt, jul[k], yl,
                diag if out else None, L.DIAG_OUT_LEVEL if out else L.DIAG_NONE)
    sh.join()
    torch.cuda.synchronize()
    idx = np.sort(np.random.default_rng(5).choice(n, 2048, replace=False))
    idx[-1] = n - 1
    st, isn = cols.state[:, idx], cols.isnow[idx]
    for k in range(nsteps):
        st, isn, dg, _ = oracle_port.step(load_params(), tuple(opts), cases.CASE_NML_ZSOIL, dt, yl,
                                          jul[k], st, isn, cols.static_f[:, idx],
                                          cols.static_i[:, idx], F[k][:, idx])
        if k == last:
            od = np.stack([dg[L.DIAG_FULL.index(m)] for m in L.DIAG_OUT if m != "T2M"])
    got = cs.state.cpu().numpy()[:, idx]
    gd = diag.cpu().numpy()[:, idx]
    gd = np.stack([gd[i] for i, m in enumerate(L.DIAG_OUT) if m != "T2M"])
    assert np.array_equal(cs.isnow.cpu().numpy()[idx], isn)
    ok = bit_equal(got, st).all(0) & bit_equal(gd, od).all(0)
    assert ok.all(), f"{(~ok).sum()} of {idx.size} sampled columns differ"


@pytest.mark.parametrize("variant", VARIANTS32)
@pytest.mark.parametrize("kind,opt_veg", [("mixed", 1), ("global", 2)])
def test_year_trajectory_bit_exact_vs_oracle(engines, oracle_port, kind, opt_veg, variant):
    """A whole year of hourly steps (8,784 = config #5's length) of 256 columns,
    bit for bit against the fp32 C restatement (itself bit-exact to the
    reference on every fixture): state, ISNOW and the output fluxes compared
    after each of 12 chunks of 732 steps (nmp_run on the GPU, the library's
    own time loop on the CPU; both form JULIAN = julian0 + s*dt/86400 in
    float from the same chunk start).  Covers slow dynamics that the short
    fixtures cannot: snowpack build-up and melt, soil freezing, phenology
    through the seasons and (opt_veg 2) the carbon pools."""
    from noahmp_amd.engine import ColumnState
    from noahmp_amd.params import Params
    P = Params.builtin()
    opts = dict(L.CASE_NML_OPTIONS, opt_veg=opt_veg)
    otuple = tuple(opts[k] for k in L.OPTION_NAMES)
    eng = engines(otuple, 4, variant=variant)
    n, dt, nsteps, nchunk, yl = 256, 3600.0, 8784, 12, 366
    cols = cases.make_columns(n, kind, P.as_dict(), seed=29, julian=0.0)
    F = np.stack([cases.forcing_step(cols, s * dt / 86400.0, yl, s, seed=29) for s in range(nsteps)])
    cs = ColumnState.from_host(cols, DEV, torch.float32)
    Fg = torch.as_tensor(F, device=DEV)
    diag = torch.zeros((L.NDIAG_OUT, n), device=DEV)
    st, isn = cols.state.copy(), cols.isnow.copy()
    per = nsteps // nchunk
    for c in range(nchunk):
        s0 = c * per
        jul0 = float(np.float32(s0 * dt / 86400.0))
        eng.run(cs, Fg[s0:s0 + per], cases.CASE_NML_ZSOIL, dt, jul0, yl, per, diag,
                L.DIAG_OUT_LEVEL)
        st, isn, dg, _ = oracle_port.run(load_params(), otuple, cases.CASE_NML_ZSOIL, dt, yl, jul0,
                                         st, isn, cols.static_f, cols.static_i, F[s0:s0 + per], per)
        torch.cuda.synchronize()
        got = cs.state.cpu().numpy()
        gd = diag.cpu().numpy()
        od = np.stack([dg[L.DIAG_FULL.index(m)] for m in L.DIAG_OUT if m != "T2M"])
        gd = np.stack([gd[i] for i, m in enumerate(L.DIAG_OUT) if m != "T2M"])
        assert np.array_equal(cs.isnow.cpu().numpy(), isn), f"chunk {c}: ISNOW differs"
        ok = bit_equal(got, st).all(0) & bit_equal(gd, od).all(0)
        assert ok.all(), f"chunk {c} (step {s0 + per}): {(~ok).sum()} of {n} columns differ"
    # the year exercised the slow processes the test is for
    snow = (cols.isnow < 0) | (isn < 0)
    assert snow.any()
    # Non-finite values only where the reference itself makes them (H13): with
    # opt_veg 2 the carbon pools of types 26/27 (Lava, White Sand: all-zero
    # carbon parameters) turn NaN in the first step; the GPU matches NaN for NaN.
    bad = ~np.isfinite(st)
    if opt_veg == 2:
        vt = cols.static_i[L.STATIC_I.index("VEGTYP")]
        pools = [L.STATE_OFF[m][0] for m in ("LFMASS", "STBLCP", "FASTCP")]
        assert bad[pools][:, np.isin(vt, (26, 27))].all()
        bad[np.ix_(pools, np.isin(vt, (26, 27)))] = False
    assert not bad.any()


@pytest.mark.parametrize("fwet,variant", [(1e-30, "casenml"), (1e-7, "casenml"),
                                          (1e-30, "generic"), (1e-30, "crs2"),
                                          (1e-30, "veg2")])
def test_tiny_canopy_wet_fraction_bit_exact(engines, oracle_port, fwet, variant):
    """Columns with a canopy wet fraction of 1e-30 or 1e-7 (FWET*VAIE, a
    numerator of the canopy Newton loop, far below its usual range) match the C
    restatement bit for bit, as every untouched column does.  (Round 3 used it
    to push the removed fast division out of its guarded range.)  Variants: the
    case.nml option-set kernel, the run-time-options kernel (option set 0
    forced), Jarvis canopy resistance (opt_crs 2, set 0) and opt_veg 2 (set 2)."""
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.params import Params
    P = Params.builtin()
    o = dict(L.CASE_NML_OPTIONS)
    if variant == "crs2":
        o["opt_crs"] = 2
    if variant == "veg2":
        o["opt_veg"] = 2
    opts = [o[k] for k in L.OPTION_NAMES]
    if variant == "generic":
        eng = Engine(P, o, device=0, precision=4)
        assert eng.option_set(0) == 0
    else:
        eng = engines(opts)
    n = 4096
    cols = cases.make_columns(n, "mixed", P.as_dict(), seed=21, julian=180.0)
    st = cols.state.copy()
    hit = np.arange(n) % 3 == 0
    st[L.s("FWET").start, hit] = np.float32(fwet)
    cols = dataclasses.replace(cols, state=st)
    f = cases.forcing_step(cols, 180.3, 366, 0, seed=21)
    cs = ColumnState.from_host(cols, DEV)
    diag = torch.zeros((L.NDIAG_FULL, n), device=DEV)
    eng.step(cs, torch.as_tensor(f, device=DEV), cases.CASE_NML_ZSOIL, 1800.0, 180.3, 366, diag,
             L.DIAG_FULL_LEVEL)
    torch.cuda.synchronize()
    est, eisn, edg, estat = oracle_port.step(load_params(), tuple(opts), cases.CASE_NML_ZSOIL, 1800.0,
                                             366, 180.3, st, cols.isnow, cols.static_f,
                                             cols.static_i, f)
    got, gd = cs.state.cpu().numpy(), diag.cpu().numpy()
    ok = bit_equal(got, est).all(0) & bit_equal(gd, edg).all(0)
    assert ok.all(), f"{(~ok).sum()} columns differ ({int((~ok & hit).sum())} of them pushed)"
    assert np.array_equal(cs.isnow.cpu().numpy(), eisn)


@pytest.mark.parametrize("level", ["none", "full"])
@pytest.mark.parametrize("variant", VARIANTS32)
@pytest.mark.parametrize("perturb", ["wind", "pressure", "fwet", "co2", "eah", "mixed"])
def test_canopy_division_domain_fallback_bit_exact(engines, oracle_port, perturb, variant, level):
    """The canopy Newton loop divides with the short exact sequence inside the
    range proof's domain (csrc/vege_domain.h, tools/div_proof.py) and falls
    back to IEEE division for a lane outside it.  Columns pushed outside the
    domain -- wind of 150-400 m/s, surface pressure of 2.5e4 Pa, a canopy wet
    fraction of 1e-20, or all three on different columns -- next to untouched
    ones: every column equals the C restatement bit for bit, in both
    occupancy instantiations.  CO2 = 0.5 Pa and EAH = 1e-5 Pa stay inside the
    canopy loop's domain but leave the stomata bisection's, which then
    divides with IEEE division alone.  At diagnostics level NONE (the 2-m
    chain skipped) the state alone is compared."""
    P = __import__("noahmp_amd.params", fromlist=["Params"]).Params.builtin()
    from noahmp_amd.engine import ColumnState
    opts = [L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES]
    eng = engines(opts, variant=variant)
    n = 4096
    cols = cases.make_columns(n, "mixed", P.as_dict(), seed=31, julian=180.0)
    f = cases.forcing_step(cols, 180.3, 366, 0, seed=31).copy()
    st = cols.state.copy()
    rng = np.random.default_rng(7)
    hit = np.arange(n) % 3 == 0
    kinds = {"wind": [0], "pressure": [1], "fwet": [2], "co2": [3], "eah": [4],
             "mixed": [0, 1, 2, 3, 4]}[perturb]
    which = np.where(hit, rng.choice(kinds, n), -1)
    fi = L.FORCING.index
    f[fi("UU"), which == 0] = rng.uniform(150.0, 400.0, (which == 0).sum()).astype(np.float32)
    f[fi("SFCPRS"), which == 1] = np.float32(2.5e4)
    f[fi("PSFC"), which == 1] = np.float32(2.5e4)
    st[L.s("FWET").start, which == 2] = np.float32(1e-20)
    # outside the stomata bisection's domain only (its divisions go IEEE)
    f[fi("CO2AIR"), which == 3] = np.float32(0.5)
    st[L.s("EAH").start, which == 4] = np.float32(1e-5)
    cols = dataclasses.replace(cols, state=st)
    cs = ColumnState.from_host(cols, DEV)
    diag = torch.zeros((L.NDIAG_FULL, n), device=DEV)
    if level == "full":
        eng.step(cs, torch.as_tensor(f, device=DEV), cases.CASE_NML_ZSOIL, 1800.0, 180.3, 366,
                 diag, L.DIAG_FULL_LEVEL)
    else:
        eng.step(cs, torch.as_tensor(f, device=DEV), cases.CASE_NML_ZSOIL, 1800.0, 180.3, 366)
    torch.cuda.synchronize()
    est, eisn, edg, _ = oracle_port.step(load_params(), tuple(opts), cases.CASE_NML_ZSOIL, 1800.0,
                                         366, 180.3, st, cols.isnow, cols.static_f, cols.static_i, f)
    got, gd = cs.state.cpu().numpy(), diag.cpu().numpy()
    ok = bit_equal(got, est).all(0)
    if level == "full":
        ok &= bit_equal(gd, edg).all(0)
    assert ok.all(), f"{(~ok).sum()} columns differ ({int((~ok & hit).sum())} of them perturbed)"
    assert np.array_equal(cs.isnow.cpu().numpy(), eisn)


def test_midloop_domain_exit_bit_exact():
    """lanes that leave the range proof's domain PART WAY through
    the canopy / bare Newton loops (after the fast loop changed TV, TAH, EAH,
    QSFC and the stomata outputs) re-run the loop with IEEE division from
    restored inputs.  The probe library (__graft_entry__._build_probe_midloop:
    the shipped sources with the TV / TGB / RAHG windows narrowed and a
    fallback counter) must equal the C restatement bit for bit on both
    occupancy kernels at diagnostics levels NONE and FULL, with the in-loop
    windows firing (tests/probe_midloop.py, run in a child process because it
    loads a second engine library)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = os.path.join(root, "noahmp-1_amd", "lib", "variants", "lib_probe_midloop.so")
    if not os.path.exists(probe):
        pytest.fail(f"probe library missing ({probe}): run __graft_entry__.build()")
    env = dict(os.environ, NOAHMP_ENGINE_LIB=probe)
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "probe_midloop.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, f"probe produced no result (rc {r.returncode}): {r.stderr[-2000:]}"
    res = json.loads(line[-1])
    for run in res["runs"]:
        print(run)
    assert r.returncode == 0 and res["ok"], res


@pytest.mark.parametrize("cfg", ["cfg5", "cfg3"])
def test_full_size_year_sample_vs_reference(engines, cfg):
    """A whole year on the product path at BASELINE size, in fp32: config #5's
    grid (1,036,800 global columns, opt_veg 2: carbon on, 8,784 steps of
    3,600 s) or config #3's set (1,048,576 mixed columns, opt_veg 1, 17,568
    steps of 1,800 s), through the bench's two stream ranges, the forcing
    generated on the device before each range's launch (nmp_forcing_synth),
    the 16 output fluxes every step.  512 seeded columns are re-run through
    the reference Fortran itself (oracle/_ref: ref_sflx_run, the time loop in
    the harness, JULIAN formed there as julian0 + s*dt/86400 in default real)
    with the forcing the device generated for them: their state and ISNOW
    after each of 12 chunks, and each chunk's last output fluxes, equal the
    reference's bit for bit.  The year tests at 256 columns cover the physics;
    this one the launch at BASELINE size for a whole year."""
    import ref
    from noahmp_amd.engine import ColumnState, StreamShards
    from noahmp_amd.params import Params
    if not ref.available():
        pytest.skip("reference oracle not built (oracle/_ref)")
    P = Params.builtin()
    kind, opt_veg, n, dt, nsteps = {"cfg5": ("global", 2, 1_036_800, 3600.0, 8784),
                                    "cfg3": ("mixed", 1, 1_048_576, 1800.0, 17568)}[cfg]
    opts = dict(L.CASE_NML_OPTIONS, opt_veg=opt_veg)
    otuple = tuple(opts[k] for k in L.OPTION_NAMES)
    eng = engines(otuple, 4)
    nchunk, yl, seed = 12, 366, 5
    cols = cases.make_columns(n, kind, P.as_dict(), seed=seed, julian=0.0)
    idx = np.sort(np.random.default_rng(seed).choice(n, 512, replace=False))
    cs = ColumnState.from_host(cols, DEV, torch.float32)
    clim = torch.as_tensor(cases.climate(cols), device=DEV).float().contiguous()
    F = torch.empty((2, L.NFORCING, n), device=DEV)
    diag = torch.zeros((L.NDIAG_OUT, n), device=DEV)
    per = nsteps // nchunk
    Fs = torch.empty((per, L.NFORCING, idx.size), device=DEV)
    idx_dev = torch.as_tensor(idx, device=DEV)
    ranges = StreamShards(eng, cs, 2)
    ref.configure(otuple)
    rec = ref.Records(cols.state[:, idx], cols.isnow[idx], cols.static_f[:, idx],
                      cols.static_i[:, idx], np.zeros((1, L.NFORCING, idx.size), np.float32))
    f32 = np.float32
    cur = torch.cuda.current_stream()
    for c in range(nchunk):
        s0 = c * per
        jul0 = f32(s0 * dt / 86400.0)
        for s in range(per):
            jul = jul0 + f32(s) * f32(dt) / f32(86400.0)   # the harness's expression
            f = F[(s0 + s) % 2]
            pre = lambda st, rng, f=f, jul=jul, k=s0 + s: eng.forcing_synth(  # noqa: E731
                clim, float(jul), yl, seed, k, f, stream=st, cols=rng)
            ranges.step(f, cases.CASE_NML_ZSOIL, dt, float(jul), yl, diag, L.DIAG_OUT_LEVEL,
                        pre=pre)
            ranges.join(cur)
            torch.index_select(f, 1, idx_dev, out=Fs[s])
        torch.cuda.synchronize()
        rec.fc = np.ascontiguousarray(Fs.cpu().numpy().transpose(0, 2, 1))
        ref.run(cases.CASE_NML_ZSOIL, dt, yl, float(jul0), rec, per)
        got = cs.state.cpu().numpy()[:, idx]
        gd = diag.cpu().numpy()[:, idx]
        want_d = rec.dg.T
        od = np.stack([want_d[L.DIAG_FULL.index(m)] for m in L.DIAG_OUT if m != "T2M"])
        gd = np.stack([gd[i] for i, m in enumerate(L.DIAG_OUT) if m != "T2M"])
        assert np.array_equal(cs.isnow.cpu().numpy()[idx], rec.isn), f"chunk {c}: ISNOW differs"
        ok = bit_equal(got, rec.st.T).all(0) & bit_equal(gd, od).all(0)
        assert ok.all(), f"chunk {c} (step {s0 + per}): {(~ok).sum()} of {idx.size} columns differ"
    assert (rec.isn < 0).any() or (cols.isnow[idx] < 0).any()  # snow came and went
