"""Diagnostic (GPU box): the stream-shard scenario of
tests/test_gpu_parity.py::test_stream_shards_equal_single_launch, step by
step, for the library NOAHMP_ENGINE_LIB names (round 3: the guarded
fast-division builds of commit 5cd66f0 with -DNMP_FAST_DIV/-DNMP_DIV_GUARD
variants, since removed -- profiles/r03/fdiv_shard_diag_*.txt).  After each step the sharded
and single-launch states are compared; on the first difference both are
compared with the C restatement (oracle, checker only) stepped from the same
start state, and the differing columns are listed with their fields.
python tools/fdiv_shard_diag.py [nshards]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import conftest  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402
from golden_io import bit_equal, load_params  # noqa: E402

import port  # noqa: E402  (oracle: the checker only)


def redo(reset):
    import ctypes as C
    from noahmp_amd import lib
    v = C.c_ulonglong(0)
    f = getattr(lib.load(), "nmp_div_redo_count", None)  # (the removed fast-division builds)
    if f is None:
        return None
    rc = f(C.byref(v), int(reset))
    return int(v.value) if rc == 0 else None


def main():
    from noahmp_amd import cases, layout as L
    from noahmp_amd.engine import ColumnState, Engine, StreamShards
    from noahmp_amd.params import Params
    nsh = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n, dev = 200_003, "cuda:0"
    opts = [L.CASE_NML_OPTIONS[k] for k in L.OPTION_NAMES]
    eng = Engine(Params.builtin(), L.CASE_NML_OPTIONS, device=0, precision=4)
    cols = cases.make_columns(n, "mixed", Params.builtin().as_dict(), seed=6, julian=200.0)
    a = ColumnState.from_host(cols, dev)
    b = ColumnState.from_host(cols, dev)
    sh = StreamShards(eng, a, nsh)
    for s in range(6):
        jul = 200.0 + s / 48.0
        f = cases.forcing_step(cols, jul, 365, s, seed=6)
        F = torch.as_tensor(f, device=dev)
        st0, isn0 = b.state.cpu().numpy().copy(), b.isnow.cpu().numpy().copy()
        redo(True)
        sh.step(F, cases.CASE_NML_ZSOIL, 1800.0, jul, 365, None, L.DIAG_NONE)
        sh.join()
        torch.cuda.synchronize()
        ra = redo(True)
        eng.step(b, F, cases.CASE_NML_ZSOIL, 1800.0, jul, 365)
        torch.cuda.synchronize()
        rb = redo(True)
        print(f"step {s}: re-run column-steps sharded {ra}, single {rb}", flush=True)
        sa, sb = a.state.cpu().numpy(), b.state.cpu().numpy()
        diff = ~bit_equal(sa, sb).all(0)
        print(f"step {s}: {int(diff.sum())} columns differ", flush=True)
        if diff.any():
            idx = np.nonzero(diff)[0]
            sub = lambda x: x[:, idx] if x.ndim == 2 else x[idx]
            est, eisn, _, _ = port.step(load_params(), tuple(opts), cases.CASE_NML_ZSOIL, 1800.0,
                                        365, jul, sub(st0), sub(isn0), sub(cols.static_f),
                                        sub(cols.static_i), sub(f))
            oka = bit_equal(sa[:, idx], est).all(0)
            okb = bit_equal(sb[:, idx], est).all(0)
            print(f"  vs oracle: sharded ok {int(oka.sum())}/{idx.size}, single ok "
                  f"{int(okb.sum())}/{idx.size}")
            for j, c in enumerate(idx[:6]):
                bad = np.nonzero(~bit_equal(sa[:, c:c + 1], sb[:, c:c + 1])[:, 0])[0]
                print(f"  column {c} (wave {c // 64} lane {c % 64}): fields {bad.tolist()[:12]}")
                for k in bad[:6]:
                    print(f"    [{k}] sharded {sa[k, c]!r} single {sb[k, c]!r} oracle {est[k, j]!r}")
            return 1
    print("all steps identical")
    return 0


if __name__ == "__main__":
    sys.exit(main())
