"""The bench's CPU-baseline leg (oracle/cpu_baseline.py): forked single-core
workers step strided samples of the column set through the reference (or the
C restatement) and the line reports the wall-clock rate.  Small sizes, CPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import noahmp_pkg  # noqa: E402,F401


def test_workers_take_strided_samples(monkeypatch):
    """Worker i of W steps columns i, i+W, i+2W, ...: each sample spans the
    whole (coherently ordered) set instead of one latitude band."""
    import cpu_baseline
    from noahmp_amd import cases, layout as L
    from noahmp_amd.params import Params
    pd = Params.builtin().as_dict()
    cols = cases.make_columns(1024, "mixed", pd, seed=4, julian=180.0)
    taken = []
    real_take = type(cols).take

    def spy(self, idx):
        taken.append(np.asarray(idx).copy())
        return real_take(self, idx)
    monkeypatch.setattr(type(cols), "take", spy)
    cpu_baseline._CTX.update(cols=cols, params=pd, options=L.options_tuple(L.CASE_NML_OPTIONS),
                             zsoil=np.asarray(cases.CASE_NML_ZSOIL, np.float32), dt=1800.0,
                             julian0=180.0, yearlen=366, seed=4, period=4)
    # in-process call of the worker body (no fork), kind "port", 2 steps
    import port
    if not port.available(4):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "port"], check=True)
    cpu = sorted(os.sched_getaffinity(0))[0]
    el = cpu_baseline._worker((1, 4, cpu, "port", 64, 2, 0.0, 4))
    assert el > 0
    assert np.array_equal(taken[0], np.arange(1, 4 * 64, 4))


def test_measure_reports_a_rate():
    import cpu_baseline
    from noahmp_amd import cases, layout as L
    from noahmp_amd.params import Params
    pd = Params.builtin().as_dict()
    cols = cases.make_columns(2048, "mixed", pd, seed=5, julian=180.0)
    r = cpu_baseline.measure(cols, pd, L.options_tuple(L.CASE_NML_OPTIONS), cases.CASE_NML_ZSOIL,
                             1800.0, 180.0, 366, 5, 4, workers=2, cols_per_worker=256, nsteps=2)
    # cores: at most the 2 asked for (fewer where this job may use fewer CPUs)
    assert r["value"] > 0 and 1 <= r["cores"] <= 2 and r["unit"] == "column-steps/s"
    assert r["kind"] in ("reference", "port")
    assert f"stride {r['cores']} " in r["sample"]
