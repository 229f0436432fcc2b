#!/usr/bin/env python3
"""Headline benchmark: land-column time steps per second (noahmp_sflx on MI355X).

Workload (BASELINE.json configs[2], "config #3"): 1,048,576 synthetic columns
per GPU, 4 soil + 3 snow layers, mixed vegetated USGS types / soil types /
soil colours, ISNOW uniform in {0,-1,-2,-3}, dynamic vegetation off
(case.nml options), fp32.  The columns are laid out in the engine's coherent
order (noahmp_amd/order.py: 4-degree longitude band, snow or not, vegetation
type -- the order the offline driver gives a grid's land points); --order
as-generated keeps the generator's shuffled order, the worst case.  One bench step = one noahmp_sflx time step of
every column (one kernel launch, state resident in HBM); every
--out-every'th step also writes the 16 output diagnostics and, for N > 1,
all-gathers them to every rank (north_star's single RCCL all-gather over
xGMI, --gather all; or gathers them to rank 0 only, the writing rank, with
--gather root) on a side stream.

Multi-GPU: one process per GPU, columns statically sharded with no data-path
collective other than that diagnostics gather; per-GPU work is fixed (weak
scaling).  `--gpus N` under torchrun (WORLD_SIZE = N) runs as that launcher's
rank; without a launcher bench.py starts the N rank processes itself
(`spawn_ranks`, before anything touches the GPU) and exits non-zero if any
rank fails or WORLD_SIZE disagrees with --gpus -- it never measures one GPU
under an N-GPU label.

Prints one JSON line (rank 0) with the driver contract fields plus
`roofline` (dominant kernel vs HBM peak) and `cpu_baseline`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L, shard  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
# VALU issue peak: 256 CUs x 4 SIMD-32 x 2.4 GHz / 2 cycles per wave64 instruction
# (MI355X_MICROARCH.md, "Wave scheduling"; f64 and transcendental instructions take
# longer, so the fraction below is a lower bound on the VALU pipe's busy share)
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2
SIMDS, CLOCK_GHZ = 256 * 4, 2.39  # the kernel holds 2.39 GHz (profiles/r02/clock.txt)
# SIMD cycles per wave64 VALU instruction by class (MI355X_MICROARCH.md constants
# table: v_fma_f32 2 cyc on a SIMD-32; the vector fp64 rate is half the fp32 rate;
# v_exp/v_log/v_rcp/v_sqrt issue at a quarter of the fp32 rate); every other VALU
# instruction (moves, selects, compares, integer, conversions) at the fp32 rate
VALU_CYCLES = {"f32": 2, "f64": 4, "trans_f32": 8, "trans_f64": 16, "other": 2}


def valu_weighted(tj: dict, launches: int, step_ms: float):
    """Cycle-weighted VALU busy share of the chip: sum over
    the instruction classes of (count x SIMD cycles per wave64 instruction),
    per step, over (SIMDs x clock x GPU step time).  Counts from the PMC
    passes in profiles/traffic.json (per dispatch)."""
    k = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
         "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_ADD_F64",
         "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64")
    if not all(x in tj for x in k):
        return None
    f32 = sum(tj[f"SQ_INSTS_VALU_{o}_F32"] for o in ("ADD", "MUL", "FMA"))
    f64 = sum(tj[f"SQ_INSTS_VALU_{o}_F64"] for o in ("ADD", "MUL", "FMA"))
    t32, t64 = tj["SQ_INSTS_VALU_TRANS_F32"], tj.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
    other = tj["SQ_INSTS_VALU"] - f32 - f64 - t32 - t64
    cls = {"f32": f32, "f64": f64, "trans_f32": t32, "trans_f64": t64, "other": other}
    cyc = sum(cls[c] * VALU_CYCLES[c] for c in cls) * launches
    avail = SIMDS * CLOCK_GHZ * 1e9 * step_ms * 1e-3
    out = {"weighted": cyc / avail, "cycles_per_class": VALU_CYCLES,
           "insts_per_wave": {c: v / tj["SQ_WAVES"] for c, v in cls.items()},
           "simd_cycles_per_step": cyc, "simd_cycles_available": avail}
    if "SQ_ACTIVE_INST_VALU" in tj:
        # quad-cycles (MI355X_MICROARCH.md: SQ_ACTIVE_INST_* count quad-cycles),
        # summed over waves: overlapping waves count separately, so it can
        # exceed the SIMDs' cycles -- reported raw, not as a pipe share
        out["active_inst_valu_per_simd_cycle"] = (4 * tj["SQ_ACTIVE_INST_VALU"] * launches
                                                  / avail)
    if "lane_util" in tj:
        # share of the 64 lanes doing useful work in the VALU cycles the waves
        # issue (SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU), one PMC pass):
        # masked-off lanes (divergence, Newton loops running their wave's
        # slowest lane) are the difference to 1
        out["lane_util"] = tj["lane_util"]
    return out
METRIC = BASELINE_METRIC = "land-columns·timesteps/sec at 4 soil + 3 snow layers, 1/2/4/8 MI355X"


def bytes_per_colstep(precision: int, diag: bool) -> int:
    """Algorithmic HBM bytes per column-step: state read+write
    (56 reals + int32 ISNOW), static 6 reals + 6 int32, forcing 12 reals,
    + 16 output diagnostics on output steps.  fp32: 552 (+64)."""
    s = precision
    b = 2 * (56 * s + 4) + 6 * s + 6 * 4 + 12 * s
    return b + (16 * s if diag else 0)


def workload_name(a, n: int) -> str:
    """BASELINE.json config this run corresponds to, else a plain description."""
    veg = "dynamic_veg + carbon on" if a.opt_veg in (2, 5) else "dynamic_veg off"
    if n == 1 << 20 and a.kind == "mixed" and a.precision == 4 and a.opt_veg == 1:
        return ("config #3: 1,048,576 columns/GPU, 4 soil + 3 snow layers, dynamic_veg off, "
                "case.nml options")
    if n == 65536 and a.kind == "casenml" and a.precision == 8:
        return "config #2: 65,536 replicated case.nml columns, 4 soil / 0 snow layers, fp64"
    if a.kind == "global" and a.precision == 8 and a.opt_veg == 2:
        return (f"config #5 per GPU: {n} columns of the 0.25-degree global grid, "
                f"{veg}, fp64, output every {a.out_every} step(s)")
    if a.kind == "conus":
        return f"config #4 per GPU: {n} CONUS-like columns (all USGS/STAS types), {veg}"
    return f"{n} {a.kind} columns/GPU, 4 soil + 3 snow layers, {veg}"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--ncol", type=int, default=1 << 20, help="columns per GPU")
    ap.add_argument("--kind", default="mixed", choices=("mixed", "conus", "casenml", "global"),
                    help="column set: mixed (config #3), conus (config #4 types), casenml "
                         "(replicated run/case.nml column, config #2), global (0.25-degree "
                         "grid order, config #5)")
    ap.add_argument("--opt-veg", type=int, default=1,
                    help="dynamic vegetation option (2 = carbon model on, config #5)")
    ap.add_argument("--precision", type=int, default=4, choices=(4, 8))
    ap.add_argument("--math", default="ref", choices=("ref", "fast"))
    ap.add_argument("--dt", type=float, default=1800.0)
    ap.add_argument("--out-every", type=int, default=6,
                    help="output (diag + all-gather) step interval; default 6 = run/case.nml's "
                         "output_frequency '3 hour' at the bench's 1800-s step")
    ap.add_argument("--gather", default="all", choices=("root", "all"),
                    help="output-step diagnostics collective for N > 1: 'all' (default) "
                         "all-gathers to every rank, north_star's single RCCL all-gather over "
                         "xGMI at output steps; 'root' gathers to rank 0 only, the rank that "
                         "writes LDASOUT (what the offline driver does)")
    ap.add_argument("--gather-dtype", default="native", choices=("native", "f32"),
                    help="type of the gathered fluxes for N > 1: the engine's ('native'), or "
                         "f32 (the reference's output precision: half the link bytes of an "
                         "fp64 run; the state stays fp64)")
    ap.add_argument("--period", type=int, default=48, help="resident forcing slices (cycled)")
    ap.add_argument("--forcing", default="resident", choices=("resident", "device"),
                    help="resident: --period host-generated forcing slices held in HBM and "
                         "cycled; device: every step's forcing generated on the device "
                         "(nmp_forcing_synth, counter-based hash) on each range's stream just "
                         "before its launch -- the long-run path (config #5, SURVEY 8d)")
    ap.add_argument("--streams", type=int, default=2,
                    help="column ranges stepped on their own HIP streams (overlaps launch tails)")
    ap.add_argument("--order", default="lon-snow-type",
                    choices=("as-generated", "lon", "lon-type", "lon-snow-type",
                             "lon-snow-type-soil"),
                    help="column order on the GPU (columns are independent: any permutation "
                         "gives bit-identical per-column results); 'lon' groups columns of "
                         "similar solar time into the same wave, like a real lat-lon grid")
    ap.add_argument("--order-band", type=float, default=None,
                    help="longitude band (degrees) of the coherent column orders; default 4, "
                         "32 for the conus kind (its 27 types leave few columns per key in a "
                         "524,288-column shard: +4.6 %%, DESIGN.md \"Launch size and config "
                         "#4's shard\")")
    ap.add_argument("--rebin-tile", type=int, default=0,
                    help="column re-binning (nmp_rebin): sort columns by the previous step's "
                         "vege_flux trip count within tiles of this many columns (0 = off)")
    ap.add_argument("--rebin-every", type=int, default=1, help="re-sort every this many steps")
    ap.add_argument("--cpw", type=int, default=0,
                    help="columns per wave (8..64, multiple of 8); 0 = the engine's automatic "
                         "choice (fewer per wave when the column set cannot fill the chip)")
    ap.add_argument("--emulate-rank", type=int, default=None,
                    help="(N = 1 only) step the column block rank R of an N-GPU run holds "
                         "(seed 1000 + R, first global column R * ncol): the shards of a "
                         "multi-GPU run measured one at a time on one GPU")
    ap.add_argument("--force-collective", action="store_true",
                    help="(under a launcher, world 1) issue the output-step collective even "
                         "though one rank has nothing to exchange: the RCCL code path's own "
                         "cost on the GPU (its copy kernels), measurable on one GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=32)
    ap.add_argument("--launch-probe", action="store_true",
                    help="launcher check only (CPU tests): every rank joins the process group "
                         "over gloo and contributes its column count, rank 0 prints the line "
                         "with n_gpus and the summed columns; no GPU is touched, no rate")
    ap.add_argument("--stagger", action="store_true",
                    help="start the stream ranges out of phase (the second range's first "
                         "step waits for the first range's first launch)")
    ap.add_argument("--first-range", type=float, default=None,
                    help="(launch-size study) the first of two stream ranges' share of the "
                         "columns; default equal ranges")
    ap.add_argument("--launch-cols", type=int, default=0,
                    help="(launch-size study) step each stream's column range as sequential "
                         "launches of at most this many columns (0 = one launch per range)")
    ap.add_argument("--replicate", type=int, default=1,
                    help="(launch-size study) generate ncol/R columns, order them, and tile "
                         "the ordered set R times: the waves of a small set in a large launch")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-measured HBM bytes per launch (written by tools/pmc_traffic.py)")
    a = ap.parse_args()
    if a.order_band is None:
        a.order_band = 32.0 if a.kind == "conus" else 4.0
    return a


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, check_gpus: bool = True) -> int:
    """`bench.py --gpus N` started without a launcher: start N rank processes
    of this same command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one
    per GPU, rendezvous on 127.0.0.1) and return the job's exit status.  This
    process never touches the GPU (it only counts devices), so the ranks are
    children, not an exec.  Any rank failing fails the job: the others are
    stopped and the status is non-zero -- never a silent one-GPU line."""
    import signal
    import subprocess
    backend = os.environ.get("NMP_BENCH_BACKEND", "nccl")
    if backend == "nccl" and check_gpus:
        import torch  # device_count() does not initialise the GPU on this image
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs for RCCL, {have} found",
                  file=sys.stderr, flush=True)
            return 2
    port = os.environ.get("MASTER_PORT") or str(_free_port())

    def die_with_parent():
        # in the child, before exec (nothing has touched the GPU): the kernel
        # sends SIGTERM to the rank if this launcher dies, even by SIGKILL
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG

    procs, live = [], []

    def stop(sig=signal.SIGTERM):
        for q in live:
            try:
                os.killpg(q.pid, sig)
            except ProcessLookupError:
                pass

    def forward(signum, _frame):
        # a signal to the launcher reaches the ranks too (they run in their own
        # sessions, so a terminal's Ctrl-C or a driver's SIGTERM would not)
        stop(signum)
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)}
    status = 0
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                       NMP_BENCH_SPAWNED="1")
            p = subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                 env=env, start_new_session=True, preexec_fn=die_with_parent)
            procs.append(p)
            live.append(p)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"bench.py: rank {procs.index(p)} exited with {rc}; stopping the job",
                          file=sys.stderr, flush=True)
                    stop()  # a rank blocked in a collective would wait forever
            time.sleep(0.05)
    finally:
        # any exit path (a signal, an exception, a caller's timeout) takes the
        # ranks down with it: none may outlive the job holding the GPU
        stop()
        for q in live:
            try:
                q.wait(timeout=10)
            except subprocess.TimeoutExpired:
                stop(signal.SIGKILL)
        for s_, h in old.items():
            signal.signal(s_, h)
    return status


def launch_probe(a, world: int, rank: int, use_dist: bool):
    """--launch-probe: the rank layout and rendezvous of a run, without the GPU.
    Each rank builds its column block (the same generator call as a run) and the
    ranks all-reduce (count, first global column index) over gloo."""
    import torch
    import torch.distributed as dist
    from noahmp_amd.params import Params
    cols = cases.make_columns(a.ncol, a.kind, Params.builtin("STAS", "USGS").as_dict(),
                              seed=1000 + rank, julian=180.0, first=rank * a.ncol)
    t = torch.tensor([cols.isnow.shape[0], rank * a.ncol, 1], dtype=torch.int64)
    if use_dist:
        dist.init_process_group("gloo")
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "column-steps/s",
                          "n_gpus": world, "launch_probe": True, "ranks_joined": int(t[2]),
                          "ncol_total": int(t[0]), "first_col_sum": int(t[1])}), flush=True)
    if use_dist:
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, check_gpus=not a.launch_probe))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # launched by torchrun or spawn_ranks (even with one rank): the distributed path
    use_dist = "RANK" in os.environ and "MASTER_ADDR" in os.environ
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}: launch with torchrun "
              f"--nproc-per-node {a.gpus}, or without a launcher", file=sys.stderr, flush=True)
        sys.exit(2)
    if os.environ.get("NMP_BENCH_FAIL_RANK") == str(rank):  # test hook: a rank that dies
        sys.exit(3)
    if os.environ.get("NMP_BENCH_HANG_DIR"):  # test hook: ranks that never finish
        with open(os.path.join(os.environ["NMP_BENCH_HANG_DIR"], f"rank{rank}.pid"), "w") as f:
            f.write(str(os.getpid()))
        time.sleep(600)
    if a.launch_probe:
        return launch_probe(a, world, rank, use_dist)

    from noahmp_amd.params import Params
    P = Params.builtin("STAS", "USGS")
    pdict = P.as_dict()
    opt_dict = dict(L.CASE_NML_OPTIONS, opt_veg=a.opt_veg)
    options = L.options_tuple(opt_dict)
    julian0, yearlen = 180.0, 366
    if a.emulate_rank is not None and world != 1:
        print("bench.py: --emulate-rank is a one-GPU measurement", file=sys.stderr, flush=True)
        sys.exit(2)
    shard_id = rank if a.emulate_rank is None else a.emulate_rank
    seed = 1000 + shard_id
    assert a.replicate >= 1 and a.ncol % a.replicate == 0
    ngen = a.ncol // a.replicate
    cols = cases.make_columns(ngen, a.kind, pdict, seed=seed, julian=julian0,
                              first=shard_id * a.ncol)
    if a.order != "as-generated":
        from noahmp_amd.order import coherent_order
        cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, a.order,
                                        band_deg=a.order_band))
    if a.replicate > 1:
        cols = cols.take(np.tile(np.arange(ngen), a.replicate))

    # ---- CPU baseline (rank 0, N=1), BEFORE anything touches the GPU ------
    cpu = None
    if world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        try:
            import cpu_baseline
            cpu = cpu_baseline.measure(cols, pdict, options, cases.CASE_NML_ZSOIL, a.dt, julian0,
                                       yearlen, seed, a.period, nsteps=a.cpu_steps)
        except Exception as e:  # the baseline is reported, never required
            cpu = {"value": None, "error": repr(e)[:200]}

    import torch
    import torch.distributed as dist
    from noahmp_amd.engine import ColumnState, Engine, StreamShards

    # NMP_BENCH_BACKEND=gloo: rehearsal of the N>1 control flow on fewer GPUs
    # than ranks (ranks share devices, the gather is staged through the host);
    # never a measurement -- RCCL refuses two ranks on one device
    backend = os.environ.get("NMP_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dtype = torch.float32 if a.precision == 4 else torch.float64
    eng = Engine(P, opt_dict, device=local, precision=a.precision, math=a.math)
    eng.set_cols_per_wave(a.cpw)
    from noahmp_amd import lib as _nlib
    build_hash = _nlib.load().nmp_build_hash().decode()  # lib.load refuses a stale library
    cs = ColumnState.from_host(cols, dev, dtype)
    n = cs.ncol
    if a.forcing == "resident":
        F = torch.empty((a.period, L.NFORCING, n), dtype=dtype, device=dev)
        for s in range(a.period):
            F[s].copy_(torch.from_numpy(cases.forcing_step(
                cols, (julian0 + s * a.dt / 86400.0) % yearlen, yearlen, s, seed=seed)))
    else:
        # two forcing buffers: step k writes buffer k % 2 on each range's stream
        # right before that range's launch (stream order makes reuse safe)
        F = torch.empty((2, L.NFORCING, n), dtype=dtype, device=dev)
        clim = torch.as_tensor(cases.climate(cols), device=dev).to(dtype).contiguous()
    gather_dst = 0 if a.gather == "root" else None
    ranges = StreamShards(eng, cs, a.streams, rebin_tile=a.rebin_tile, rebin_every=a.rebin_every,
                          launch_cols=a.launch_cols, first_frac=a.first_range,
                          stagger=a.stagger)
    comm = torch.cuda.Stream(dev) if use_dist else None
    if use_dist:
        # after the range streams exist: RCCL's communicator creates streams of
        # its own, and created first they left the two ranges sharing one of
        # the process's hardware queues (GPU_MAX_HW_QUEUES=4), serialising them
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        # double-buffered output-step gather; a receiving rank's engine writes
        # straight into its own slot of the gather buffer (no local copy)
        gat = shard.DiagGather(L.NDIAG_OUT, world * n, dtype, dev, dst=gather_dst, comm=comm,
                               force_collective=a.force_collective,
                               wire_dtype=torch.float32 if a.gather_dtype == "f32" else None)
        sched = shard.OutputSchedule(a.out_every, gat, streams=ranges.streams)
    else:
        gat = None
        sched = shard.OutputSchedule(a.out_every, bufs=[
            torch.zeros((L.NDIAG_OUT, n), dtype=dtype, device=dev) for _ in range(2)])
    del cols

    def step(k, ev=None):
        """Bench step k: every column range on its own stream (StreamShards), plus the
        async diagnostics gather on output steps (shard.OutputSchedule)."""
        d = sched.diag_for(k)
        # day of year: the calendar wraps at yearlen (a run past the year's end
        # continues into the next year; the engine rejects julian > yearlen)
        jul = (julian0 + k * a.dt / 86400.0) % yearlen
        if a.forcing == "resident":
            f, pre = F[k % a.period], None
        else:
            f = F[k % 2]
            pre = lambda st, rng: eng.forcing_synth(  # noqa: E731
                clim, jul, yearlen, seed, k, f, first_col=shard_id * n, stream=st, cols=rng)
        ranges.step(f, cases.CASE_NML_ZSOIL, a.dt, jul, yearlen, d,
                    L.DIAG_OUT_LEVEL if d is not None else L.DIAG_NONE, events=ev, pre=pre)
        sched.finish(k, producers=ranges.producers)
        return d is not None

    for k in range(a.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(a.streams)] for _ in range(a.steps)]
    outs = 0
    t0 = time.perf_counter()
    for k in range(a.steps):
        outs += step(a.warmup + k, evs[k])
    if gat is not None:
        gat.wait_all()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # per-launch mean duration (what rocprof reports; the ranges' launches overlap)
    # and the GPU time per step: first launch start to last launch end, / steps
    kern_ms = float(np.mean([e0.elapsed_time(e1) for ev in evs for e0, e1 in ev]))
    step_ms = max(evs[0][0][0].elapsed_time(e1) for _, e1 in evs[-1]) / a.steps
    st_bad = int((cs.status != 0).sum().item())
    finite = bool(torch.isfinite(cs.state[L.s("STC")]).all().item())
    if use_dist:
        t = torch.tensor([elapsed, kern_ms, step_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, step_ms = float(t[0]), float(t[1]), float(t[2])

    if rank == 0:
        colsteps = world * n * a.steps
        value = colsteps / elapsed
        # algorithmic bytes per launch, averaged over plain and output steps
        bps = n * (bytes_per_colstep(a.precision, False) * (a.steps - outs)
                   + bytes_per_colstep(a.precision, True) * outs) / a.steps
        bpl = bps / len(ranges.ranges)
        # the S launches of a step run concurrently: rate = bytes per step / GPU time per step
        achieved = bps / (step_ms * 1e-3) / 1e9
        traffic = valu = None
        if os.path.exists(a.traffic):
            with open(a.traffic) as f:
                tj = json.load(f)
            from noahmp_amd import build as _build
            if tj.get("ncol") == n and tj.get("precision") == a.precision and \
                    tj.get("streams", 1) == len(ranges.ranges) and \
                    tj.get("math") == a.math and tj.get("kind", "mixed") == a.kind and \
                    tj.get("order", "as-generated") == a.order and \
                    (a.order == "as-generated" or tj.get("order_band", 4.0) == a.order_band) and \
                    tj.get("out_every", 2) == a.out_every and \
                    tj.get("source_hash") == _build.source_hash() \
                    and os.environ.get("NOAHMP_ENGINE_LIB") is None:
                traffic = tj.get("bytes_per_launch")
                if tj.get("SQ_INSTS_VALU"):
                    # PMC wave-instructions per launch x launches per step / GPU time per step
                    g = tj["SQ_INSTS_VALU"] * len(ranges.ranges) / (step_ms * 1e-3) / 1e9
                    valu = {"achieved": g, "peak": VALU_PEAK_GINST, "unit": "G wave-instr/s",
                            "frac": g / VALU_PEAK_GINST,
                            "insts_per_wave": tj["SQ_INSTS_VALU"] / tj["SQ_WAVES"],
                            "source": "SQ_INSTS_VALU / SQ_WAVES, rocprofv3 --pmc "
                                      "(profiles/traffic.json)"}
                    w = valu_weighted(tj, len(ranges.ranges), step_ms)
                    if w is not None:
                        valu.update(w)
        line = {
            "metric": METRIC, "value": value, "unit": "column-steps/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed * 1e3 / a.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" if a.precision == 4 else "f64",
            "data": f"synthetic (seeded {a.kind} USGS/STAS columns, diurnal forcing; no dataset)",
            "config": {"workload": workload_name(a, n), "kind": a.kind, "opt_veg": a.opt_veg,
                       "ncol_per_gpu": n,
                       "ncol_total": world * n, "dt_s": a.dt, "out_every": a.out_every,
                       "math": a.math, "column_order": a.order, "forcing": a.forcing,
                       "streams": len(ranges.ranges), "cols_per_wave": a.cpw or "auto",
                       "rebin": {"tile": a.rebin_tile, "every": a.rebin_every}
                       if a.rebin_tile else None,
                       "parallelism": f"column-shard x{world}",
                       "emulated_rank": a.emulate_rank,
                       "force_collective": a.force_collective or None,
                       "gather": a.gather if use_dist else None,
                       "gather_dtype": (a.gather_dtype if a.gather_dtype != "native" else
                                        ("f32" if a.precision == 4 else "f64"))
                       if use_dist else None,
                       "backend": backend if use_dist else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "sflx_step_kernel", "kernel_ms": kern_ms,
                         "bytes_per_launch": bpl, "launches_per_step": len(ranges.ranges),
                         "step_ms": step_ms, "bytes_per_step": bps, "valu": valu},
            "cpu_baseline": cpu,
            "checks": {"status_nonzero_cols": st_bad, "stc_finite": finite,
                       "build_hash": build_hash},
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
