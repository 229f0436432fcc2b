"""Multi-rank path on CPU (gloo, world_size 2): column sharding + the
output-step diagnostics all-gather reproduce the single-rank result bit for
bit (SURVEY.md 8e correctness test).  Per-shard physics is computed by the
oracle restatement (this is a test of the sharding plumbing)."""
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


def _worker(rank, world, port, out_path, dst=None):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle"), os.path.join(root, "tests")]
    import noahmp_pkg  # noqa: F401
    import port as oracle
    from golden_io import load, load_params
    from noahmp_amd import shard as sh
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load("single_casenml_mixed.npz")
    n = g["isnow0"].shape[0]
    s0, cnt = sh.shard_range(n, rank, world)
    sl = slice(s0, s0 + cnt)
    _, _, dg, _ = oracle.step(load_params(), tuple(g["options"]), g["zsoil"], float(g["dt"]),
                              int(g["yearlen"]), float(g["julian"]), g["state0"][:, sl],
                              g["isnow0"][sl], g["static_f"][:, sl], g["static_i"][:, sl],
                              g["forcing"][:, sl])
    idx = [L.DIAG_FULL.index(d) if d != "T2M" else L.DIAG_FULL.index("T2MV") for d in L.DIAG_OUT]
    local = torch.from_numpy(np.ascontiguousarray(dg[idx]))
    out, work = sh.gather_diag(local, async_op=True, dst=dst)
    work.wait()
    if dst is not None and rank != dst:
        assert out is None  # gather to root: only dst receives
    elif rank == (0 if dst is None else dst):
        np.save(out_path, out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dst", [None, 0, 1], ids=["all-gather", "gather-to-0", "gather-to-1"])
def test_gloo_two_rank_gather_equals_single_rank(oracle_port, tmp_path, dst):
    """All-gather (bench --gather all) and gather to one rank (the offline
    writer's and the bench's default mode) both rebuild the single-rank
    diagnostics."""
    from golden_io import load, load_params
    world, port = 2, _free_port()
    out_path = str(tmp_path / "gathered.npy")
    mp.start_processes(_worker, args=(world, port, out_path, dst), nprocs=world,
                       start_method="spawn")
    got = np.load(out_path)
    g = load("single_casenml_mixed.npz")
    _, _, dg, _ = oracle_port.step(load_params(), tuple(g["options"]), g["zsoil"],
                                   float(g["dt"]), int(g["yearlen"]), float(g["julian"]),
                                   g["state0"], g["isnow0"], g["static_f"], g["static_i"],
                                   g["forcing"])
    idx = [L.DIAG_FULL.index(d) if d != "T2M" else L.DIAG_FULL.index("T2MV") for d in L.DIAG_OUT]
    full = dg[idx]
    n = full.shape[1]
    per = n // world
    rebuilt = np.concatenate([got[r * L.NDIAG_OUT:(r + 1) * L.NDIAG_OUT] for r in range(world)],
                             axis=1)
    assert rebuilt.shape == full.shape and per * world == n
    assert np.array_equal(rebuilt, full) or np.array_equal(
        np.nan_to_num(rebuilt, nan=1e30), np.nan_to_num(full, nan=1e30))


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
