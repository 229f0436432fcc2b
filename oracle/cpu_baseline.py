"""ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.

CPU baseline leg of bench.py: times the reference Fortran noahmp_sflx
(oracle/_ref/libnoahmp_ref.so, built from /root/reference/core by
oracle/Makefile; kind "reference") -- or, when that library is absent, the C
restatement (oracle/build/liboracle_f32.so; kind "port") -- on a bounded
sample of the bench workload, on the host cores of the GPU box.

The reference is single-threaded and non-reentrant (process-global module
state, core/module_noahmp_func.f90:3854-3856), so P cores means P forked
worker processes, each stepping its own slice of columns.  Each worker is
pinned to its own PHYSICAL core (one logical CPU per core from
/proc/cpuinfo, SMT siblings left idle), so the rate is per physical core.
The time loop runs inside the library (ref_sflx_run / oracle_sflx_run): the
records are transposed into the harness layout once, before the clock starts.

Worker count: the CPUs this process may actually use -- the smallest of its
affinity set, its cgroup CPU quota and OMP_NUM_THREADS (the GPU box allots 16
CPUs per GPU and exports OMP_NUM_THREADS=16) -- one per physical core.  The
report also gives the per-core rate and the host's physical core count, so
the whole-host rate (per-core x physical cores, linear because the workers
share nothing) is stated beside the measured one.

Call this BEFORE the parent initialises the GPU (fork after HIP init is not
safe).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time

import numpy as np

_CTX = {}


def cpu_topology() -> dict[int, tuple[int, int]]:
    """logical cpu -> (physical package, core id), from /proc/cpuinfo."""
    topo, cur = {}, {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in list(f) + [""]:
                if not line.strip():
                    if "processor" in cur:
                        topo[cur["processor"]] = (cur.get("physical id", 0),
                                                  cur.get("core id", cur["processor"]))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                k = k.strip()
                if k in ("processor", "physical id", "core id"):
                    cur[k] = int(v.strip())
    except OSError:
        pass
    return topo


def physical_cores() -> int:
    topo = cpu_topology()
    return len(set(topo.values())) or (os.cpu_count() or 1)


def cgroup_cpu_quota() -> float | None:
    """CPUs granted by the cgroup (v2 cpu.max or v1 cfs quota), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def worker_cpus() -> list[int]:
    """One logical CPU per physical core of this process's affinity set, capped
    at the cgroup quota and OMP_NUM_THREADS: the CPUs the workers are pinned to."""
    aff = sorted(os.sched_getaffinity(0))
    topo = cpu_topology()
    seen, cpus = set(), []
    for c in aff:
        key = topo.get(c, (0, c))
        if key not in seen:
            seen.add(key)
            cpus.append(c)
    cap = len(cpus)
    q = cgroup_cpu_quota()
    if q is not None:
        cap = min(cap, max(1, int(q)))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        cap = min(cap, int(env))
    return cpus[:max(1, cap)]


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
    i, nw, cpu, kind, cols_per, nsteps, t_start, precision = args
    from noahmp_amd import cases  # package registered by the parent
    os.sched_setaffinity(0, {cpu})
    c = _CTX
    # every nw-th column from i: each worker's sample spans the whole column
    # set (the bench's set is in coherent order -- latitude bands, snow,
    # vegetation type -- so contiguous slices gave workers unequal work and
    # the slowest set the wall)
    cols = c["cols"].take(np.arange(i, nw * cols_per, nw))
    Fa = np.stack([cases.forcing_step(cols, c["julian0"] + s * c["dt"] / 86400.0, c["yearlen"], s,
                                      seed=c["seed"]) for s in range(min(nsteps, c["period"]))])
    if kind == "reference":
        import ref
        ref.configure(c["options"])
        rec = ref.Records(cols.state, cols.isnow, cols.static_f, cols.static_i, Fa)
        while time.time() < t_start:
            time.sleep(0.001)
        t0 = time.perf_counter()
        ref.run(c["zsoil"], c["dt"], c["yearlen"], c["julian0"], rec, nsteps)
        return time.perf_counter() - t0
    import port
    go = port.prepare_run(c["params"], c["options"], c["zsoil"], c["dt"], c["yearlen"],
                          c["julian0"], cols.state, cols.isnow, cols.static_f, cols.static_i, Fa,
                          nsteps, precision=precision)
    while time.time() < t_start:
        time.sleep(0.001)
    t0 = time.perf_counter()
    go()
    return time.perf_counter() - t0


def measure(cols, params: dict, options: tuple, zsoil, dt: float, julian0: float, yearlen: int,
            seed: int, period: int, workers: int | None = None, cols_per_worker: int = 32768,
            nsteps: int = 48) -> dict:
    """Throughput (column-steps/s) of the CPU leg over workers x cols_per_worker x nsteps."""
    import port
    import ref
    kind = "reference" if ref.available() else "port"
    if kind == "port" and not port.available(4):
        raise FileNotFoundError("no CPU baseline library: build oracle/ (make -C oracle port)")
    cpus = worker_cpus()
    if workers:
        cpus = cpus[:workers]
    workers = len(cpus)
    cols_per_worker = min(cols_per_worker, cols.n // workers)
    _CTX.update(cols=cols, params=params, options=options, zsoil=np.asarray(zsoil, np.float32),
                dt=dt, julian0=julian0, yearlen=yearlen, seed=seed, period=period)

    def timed(kind, precision):
        t_start = time.time() + 2.0 + 0.02 * workers
        with mp.get_context("fork").Pool(workers) as pool:
            el = pool.map(_worker, [(i, workers, cpus[i], kind, cols_per_worker, nsteps, t_start,
                                     precision)
                                    for i in range(workers)])
        return max(el)

    phys = physical_cores()
    wall = timed(kind, 4)
    total = workers * cols_per_worker * nsteps
    value = total / wall
    what = "Fortran reference noahmp_sflx, amdflang -O2" if kind == "reference" else \
        "C restatement -O2"
    out = {"value": value, "unit": "column-steps/s", "cores": workers, "kind": kind,
           "sample": (f"{workers} single-threaded processes, one per physical core (SMT siblings "
                      f"idle), x {cols_per_worker} columns (stride {workers} from the worker's "
                      f"index) x {nsteps} steps of the bench column set ({what}; time loop inside the library), wall {wall:.1f} s"),
           "per_core": value / workers,
           "host_physical_cores": phys,
           "whole_host_estimate": value / workers * phys,
           "whole_host_note": "per-core rate x physical cores (workers share nothing); the "
                              "measured cores are the CPUs this job may use",
           "smt": "off (one worker per physical core)",
           "cpu_model": cpu_model(), "affinity_cores": len(os.sched_getaffinity(0)),
           "cgroup_cpu_quota": cgroup_cpu_quota(),
           "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    if port.available(8):
        # fp64 leg (SURVEY 8d asks for both precisions): the C restatement in
        # double, same processes / sample (the reference itself is fp32-only, H11)
        w8 = timed("port", 8)
        out["port_f64"] = {"value": total / w8, "unit": "column-steps/s", "cores": workers,
                           "per_core": total / w8 / workers,
                           "whole_host_estimate": total / w8 / workers * phys,
                           "sample": f"C restatement fp64 -O2, same sample, wall {w8:.1f} s"}
    return out
