"""The RCCL (torch "nccl") path of the diagnostics gather on ONE GPU (run by
tests/test_gpu_driver.py in a child process, because it creates a process
group).

At world size 1 `DiagGather` normally issues no collective (nothing has to
move).  Here `force_collective=True` makes it run the multi-GPU code path on a
world-1 RCCL group: `all_gather_into_tensor` in place (dst=None) and the
gather to a root (dst=0) on a side comm stream, double-buffered, with the
bench's output loop (shard.OutputSchedule over StreamShards).  Diagnostics are
written every step, so each buffer is rewritten two steps after its
collective was issued: the comm-stream fence (`release`) must hold the next
writer back.  Every assembled output step must equal the diagnostics of a
plain run without any gather, bit for bit; `gather_diag`'s RCCL branches are
checked the same way.  The streams are created before the group, as in
bench.py.  Prints one JSON line; exit status 0 when every check passed.
"""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L, shard  # noqa: E402
from noahmp_amd.engine import ColumnState, Engine, StreamShards  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    n, nsteps, dt, yl = 65536 + 37, 6, 1800.0, 366
    P = Params.builtin()
    cols = cases.make_columns(n, "mixed", P.as_dict(), seed=5, julian=180.0)
    F = [cases.forcing_step(cols, 180.0 + k * dt / 86400.0, yl, k, seed=5) for k in range(nsteps)]
    dev = torch.device("cuda", 0)
    eng = Engine(P, L.CASE_NML_OPTIONS, device=0)

    def run(gat):
        cs = ColumnState.from_host(cols, dev)
        ranges = StreamShards(eng, cs, 2)
        if gat is None:
            bufs = [torch.zeros((L.NDIAG_OUT, n), device=dev) for _ in range(2)]
            sched = shard.OutputSchedule(1, bufs=bufs)
        else:
            sched = shard.OutputSchedule(1, gat, streams=ranges.streams)
        outs = []
        for k in range(nsteps):
            d = sched.diag_for(k)
            jul = 180.0 + k * dt / 86400.0
            ranges.step(torch.as_tensor(F[k], device=dev), cases.CASE_NML_ZSOIL, dt, jul, yl, d,
                        L.DIAG_OUT_LEVEL)
            sched.finish(k, producers=ranges.producers)
            if gat is None:
                ranges.join()
                outs.append(d.clone())
            elif k >= 1:
                # the previous output step, read while this step's collective
                # and the next writes of the other buffer are in flight
                outs.append(gat.assemble(sched.buffer(k - 1)).clone())
        if gat is not None:
            outs.append(gat.assemble(sched.buffer(nsteps - 1)).clone())
            gat.wait_all()
        torch.cuda.synchronize()
        return [o.cpu() for o in outs], cs.state.cpu()

    ref, ref_state = run(None)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0",
                      WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    res = {"backend": dist.get_backend(), "ncol": n, "steps": nsteps, "checks": {}}
    ok_all = True
    comm = torch.cuda.Stream(dev)
    for dst in (None, 0):
        gat = shard.DiagGather(L.NDIAG_OUT, n, torch.float32, dev, dst=dst, comm=comm,
                               force_collective=True)
        got, state = run(gat)
        same = [bool(torch.equal(a.view(torch.int32), b.view(torch.int32)))
                for a, b in zip(got, ref)]
        same.append(bool(torch.equal(state.view(torch.int32), ref_state.view(torch.int32))))
        issued = all(d is not None for d in gat.done)
        res["checks"][f"DiagGather dst={dst}"] = {"outputs_equal": same, "collective_ran": issued}
        ok_all &= all(same) and len(got) == nsteps and issued
    # gather_diag, both RCCL branches (all_gather_into_tensor, gather to root)
    blk = torch.randn(L.NDIAG_OUT, 4099, device=dev)
    for dst in (None, 0):
        out = shard.gather_diag(blk, dst=dst)
        torch.cuda.synchronize()
        eq = bool(torch.equal(out.view(torch.int32), blk.view(torch.int32)))
        res["checks"][f"gather_diag dst={dst}"] = eq
        ok_all &= eq
    dist.destroy_process_group()
    res["ok"] = ok_all
    print(json.dumps(res))
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
