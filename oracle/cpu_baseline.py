"""ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.

CPU baseline leg of bench.py: times the reference Fortran noahmp_sflx
(oracle/_ref/libnoahmp_ref.so, built from /root/reference/core by
oracle/Makefile; kind "reference") -- or, when that library is absent, the C
restatement (oracle/build/liboracle_f32.so; kind "port") -- on a bounded
sample of the bench workload, on the host cores of the GPU box.

The reference is single-threaded and non-reentrant (process-global module
state), so P cores means P forked worker processes, each stepping
its own slice of columns.  Call this BEFORE the parent initialises the GPU
(fork after HIP init is not safe).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time

import numpy as np

_CTX = {}


def default_workers(cap: int = 16) -> int:
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, min(n, cap))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _worker(args):
    i, kind, cols_per, nsteps, t_start, precision = args
    from noahmp_amd import cases  # package registered by the parent
    c = _CTX
    cols = c["cols"].take(np.arange(i * cols_per, (i + 1) * cols_per))
    F = [cases.forcing_step(cols, c["julian0"] + s * c["dt"] / 86400.0, c["yearlen"], s,
                            seed=c["seed"]) for s in range(min(nsteps, c["period"]))]
    st, isn = cols.state, cols.isnow
    if kind == "reference":
        import ref
        ref.configure(c["options"])
        while time.time() < t_start:
            time.sleep(0.001)
        t0 = time.perf_counter()
        for s in range(nsteps):
            st, isn, _, _ = ref.step(c["zsoil"], c["dt"], c["yearlen"],
                                     c["julian0"] + s * c["dt"] / 86400.0, st, isn,
                                     cols.static_f, cols.static_i, F[s % len(F)])
        return time.perf_counter() - t0
    import port
    Fa = np.stack(F)
    while time.time() < t_start:
        time.sleep(0.001)
    t0 = time.perf_counter()
    port.run(c["params"], c["options"], c["zsoil"], c["dt"], c["yearlen"], c["julian0"], st, isn,
             cols.static_f, cols.static_i, Fa, nsteps, precision=precision)
    return time.perf_counter() - t0


def measure(cols, params: dict, options: tuple, zsoil, dt: float, julian0: float, yearlen: int,
            seed: int, period: int, workers: int | None = None, cols_per_worker: int = 16384,
            nsteps: int = 32) -> dict:
    """Throughput (column-steps/s) of the CPU leg over workers x cols_per_worker x nsteps."""
    import port
    import ref
    kind = "reference" if ref.available() else "port"
    if kind == "port" and not port.available(4):
        raise FileNotFoundError("no CPU baseline library: build oracle/ (make -C oracle port)")
    workers = workers or default_workers()
    cols_per_worker = min(cols_per_worker, cols.n // workers)
    _CTX.update(cols=cols, params=params, options=options, zsoil=np.asarray(zsoil, np.float32),
                dt=dt, julian0=julian0, yearlen=yearlen, seed=seed, period=period)
    def timed(kind, precision):
        t_start = time.time() + 2.0 + 0.02 * workers
        with mp.get_context("fork").Pool(workers) as pool:
            el = pool.map(_worker, [(i, kind, cols_per_worker, nsteps, t_start, precision)
                                    for i in range(workers)])
        return max(el)

    wall = timed(kind, 4)
    total = workers * cols_per_worker * nsteps
    out = {"value": total / wall, "unit": "column-steps/s", "cores": workers, "kind": kind,
           "sample": (f"{workers} single-threaded processes x {cols_per_worker} columns x "
                      f"{nsteps} steps of the bench column set "
                      f"({'Fortran reference noahmp_sflx, amdflang -O2' if kind == 'reference' else 'C restatement -O2'}"
                      f"), wall {wall:.1f} s"),
           "cpu_model": cpu_model(), "affinity_cores": len(os.sched_getaffinity(0))}
    if port.available(8):
        # fp64 leg (SURVEY 8d asks for both precisions): the C restatement in
        # double, same processes / sample (the reference itself is fp32-only, H11)
        w8 = timed("port", 8)
        out["port_f64"] = {"value": total / w8, "unit": "column-steps/s", "cores": workers,
                           "sample": f"C restatement fp64 -O2, same sample, wall {w8:.1f} s"}
    return out
