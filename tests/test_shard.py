"""Multi-rank path on CPU (gloo, world sizes 2, 3 and 8, ragged shards): column
sharding + the output-step diagnostics gather reproduce the single-rank
result bit for bit (SURVEY.md 8e correctness test).  Per-shard physics is
computed by the oracle restatement (this is a test of the sharding plumbing)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import noahmp_pkg  # noqa: F401,E402  (spawned ranks re-import this module)
from noahmp_amd import layout as L, shard  # noqa: E402


def test_shard_range_partitions():
    for n in (0, 1, 7, 1024, 1000003):
        for w in (1, 2, 3, 8):
            got = [shard.shard_range(n, r, w) for r in range(w)]
            assert sum(c for _, c in got) == n
            assert all(got[r][0] + got[r][1] == got[r + 1][0] for r in range(w - 1))
            assert max(c for _, c in got) - min(c for _, c in got) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_steps(g, sl, nsteps):
    """The oracle's diagnostics (DIAG_OUT fields) after each of nsteps steps of columns sl."""
    import port as oracle
    from golden_io import load_params
    idx = [L.DIAG_FULL.index(d) if d != "T2M" else L.DIAG_FULL.index("T2MV") for d in L.DIAG_OUT]
    st, isn, out = g["state0"][:, sl], g["isnow0"][sl], []
    for k in range(nsteps):
        st, isn, dg, _ = oracle.step(load_params(), tuple(g["options"]), g["zsoil"],
                                     float(g["dt"]), int(g["yearlen"]),
                                     float(g["julian"]) + k * float(g["dt"]) / 86400.0, st, isn,
                                     g["static_f"][:, sl], g["static_i"][:, sl],
                                     g["forcing"][:, sl])
        out.append(np.ascontiguousarray(dg[idx]))
    return out


NSTEPS, OUT_EVERY = 8, 2   # 4 output steps: each of the 2 buffers is reused once


def _worker(rank, world, port, out_path, ncol, dst=None):
    """One rank of the bench/driver output loop (shard.OutputSchedule +
    DiagGather) on gloo: steps its ragged shard (oracle physics), writes each
    output step's diagnostics into the schedule's buffer, gathers them
    asynchronously, and the receiver assembles every output step."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle"), os.path.join(root, "tests")]
    import noahmp_pkg  # noqa: F401
    from golden_io import load
    from noahmp_amd import shard as sh
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load("single_casenml_mixed.npz")
    s0, cnt = sh.shard_range(ncol, rank, world)
    local = _oracle_steps(g, slice(s0, s0 + cnt), NSTEPS)
    gat = sh.DiagGather(L.NDIAG_OUT, ncol, torch.float32, "cpu", dst=dst)
    sched = sh.OutputSchedule(OUT_EVERY, gat)
    got, prev = [], None
    for k in range(NSTEPS):
        d = sched.diag_for(k)
        if d is not None:
            assert d.shape == (L.NDIAG_OUT, cnt)
            d.copy_(torch.from_numpy(local[k]))  # "the engine writes its block"
        sched.finish(k)
        if d is not None:
            if prev is not None:  # the previous output step, assembled while this one flies
                got.append(gat.assemble(prev))
            prev = sched.buffer(k)
    gat.wait_all()
    got.append(gat.assemble(prev))
    if gat.receives and rank == (0 if dst is None else dst):
        np.save(out_path, torch.stack(got).numpy())
    if not gat.receives:
        assert all(x is None for x in got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,ncol,dst", [(2, 2048, 0), (2, 2047, None), (3, 2048, 0),
                                            (3, 2047, 2), (3, 2045, None), (8, 2045, None),
                                            (8, 2043, 5)],
                         ids=["w2-even-root", "w2-ragged-all", "w3-ragged-root",
                              "w3-ragged-to-2", "w3-ragged-all", "w8-ragged-all",
                              "w8-ragged-to-5"])
def test_gloo_output_loop_equals_single_rank(oracle_port, tmp_path, world, ncol, dst):
    """SURVEY 8e correctness test of the bench/driver output loop: ragged shards
    (shard_range), double-buffered asynchronous gathers with buffer reuse, to
    one rank or to all; every output step rebuilt on the receiver equals the
    single-rank run bit for bit."""
    from golden_io import load
    port = _free_port()
    out_path = str(tmp_path / "gathered.npy")
    mp.start_processes(_worker, args=(world, port, out_path, ncol, dst), nprocs=world,
                       start_method="spawn")
    got = np.load(out_path)
    g = load("single_casenml_mixed.npz")
    full = _oracle_steps(g, slice(0, ncol), NSTEPS)
    want = np.stack([full[k] for k in range(NSTEPS) if (k + 1) % OUT_EVERY == 0])
    assert got.shape == want.shape == (NSTEPS // OUT_EVERY, L.NDIAG_OUT, ncol)
    assert np.array_equal(got.view(np.int32), want.view(np.int32))


def _wire_worker(rank, world, port, out_path):
    """A rank whose engine writes fp64 fluxes gathered as fp32 (DiagGather
    wire_dtype): two output steps through OutputSchedule, both buffers."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    import noahmp_pkg  # noqa: F401
    from noahmp_amd import shard as sh
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ncol = 1001
    s0, cnt = sh.shard_range(ncol, rank, world)
    gat = sh.DiagGather(L.NDIAG_OUT, ncol, torch.float64, "cpu", dst=None,
                        wire_dtype=torch.float32)
    sched = sh.OutputSchedule(1, gat)
    got = []
    for k in range(3):
        d = sched.diag_for(k)
        assert d.dtype == torch.float64 and d.shape == (L.NDIAG_OUT, cnt)
        vals = torch.arange(L.NDIAG_OUT * ncol, dtype=torch.float64).view(L.NDIAG_OUT, ncol)
        d.copy_(vals[:, s0:s0 + cnt] / 3.0 + k)
        sched.finish(k)
        got.append(gat.assemble(sched.buffer(k)).clone())
    gat.wait_all()
    if rank == 0:
        np.save(out_path, torch.stack(got).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_gather_fp32_wire_of_fp64_fluxes(tmp_path):
    """DiagGather(wire_dtype=float32): fp64 engine fluxes travel and arrive as
    their fp32 rounding (bench.py --gather-dtype f32), ragged shards, world 3."""
    out_path = str(tmp_path / "wire.npy")
    mp.start_processes(_wire_worker, args=(3, _free_port(), out_path), nprocs=3,
                       start_method="spawn")
    got = np.load(out_path)
    vals = np.arange(L.NDIAG_OUT * 1001, dtype=np.float64).reshape(L.NDIAG_OUT, 1001)
    want = np.stack([(vals / 3.0 + k).astype(np.float32) for k in range(3)])
    assert got.dtype == np.float32 and np.array_equal(got, want)


def _gpu_worker(rank, world, port, out_path):
    """One rank of a world-size-2 run on the box's single GPU: the HIP engine
    steps this rank's column shard; the output diagnostics are gathered over
    gloo (RCCL refuses two ranks on one device)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    import noahmp_pkg  # noqa: F401
    from golden_io import fixture_tags, load
    from noahmp_amd import cases
    from noahmp_amd import shard as sh
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.params import Params
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load("single_casenml_mixed.npz")
    n = g["isnow0"].shape[0]
    s0, cnt = sh.shard_range(n, rank, world)
    sl = slice(s0, s0 + cnt)
    eng = Engine(Params.builtin(*fixture_tags(g)), dict(zip(L.OPTION_NAMES, g["options"].tolist())),
                 device=0)
    cols = cases.ColumnSet(g["static_f"][:, sl], g["static_i"][:, sl], g["state0"][:, sl],
                           g["isnow0"][sl], *([None] * 7))
    cs = ColumnState.from_host(cols, "cuda:0")
    f = torch.as_tensor(np.ascontiguousarray(g["forcing"][:, sl]), device="cuda:0")
    diag = torch.zeros((L.NDIAG_OUT, cnt), dtype=torch.float32, device="cuda:0")
    eng.step(cs, f, g["zsoil"], float(g["dt"]), float(g["julian"]), int(g["yearlen"]), diag,
             L.DIAG_OUT_LEVEL)
    torch.cuda.synchronize()
    out = sh.gather_diag(diag.cpu())
    if rank == 0:
        np.save(out_path, out.numpy())
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_engine_shards_gather_to_reference(engine_lib, tmp_path):
    """SURVEY 8e correctness test with the HIP engine: two ranks each step
    their shard on the GPU; the gathered output fluxes equal the reference's
    single-call diagnostics bit for bit (T2M aside, a blend the reference
    does not output)."""
    from golden_io import load
    world, port = 2, _free_port()
    out_path = str(tmp_path / "gathered_gpu.npy")
    mp.start_processes(_gpu_worker, args=(world, port, out_path), nprocs=world,
                       start_method="spawn")
    got = np.load(out_path)
    g = load("single_casenml_mixed.npz")
    rebuilt = np.concatenate([got[r * L.NDIAG_OUT:(r + 1) * L.NDIAG_OUT] for r in range(world)],
                             axis=1)
    for i, name in enumerate(L.DIAG_OUT):
        if name == "T2M":
            continue
        ref = g["diag"][L.DIAG_FULL.index(name)]
        assert np.array_equal(rebuilt[i].view(np.int32), ref.astype(np.float32).view(np.int32)), \
            name
