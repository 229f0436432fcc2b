"""Diagnostic (GPU box): the fields of chosen columns of one single-call
fixture that differ from the reference, with values (NOAHMP_ENGINE_LIB picks
the library).  python tools/fdiv_cols.py combo_r2 75 89"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import conftest  # noqa: E402,F401
import numpy as np  # noqa: E402
from golden_io import fixture_tags, load  # noqa: E402
from test_gpu_parity import STATE_NAMES, run_single  # noqa: E402


def main():
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    from noahmp_amd import layout as L
    name, cols = sys.argv[1], [int(x) for x in sys.argv[2:]]
    g = load(f"single_{name}.npz")
    eng = Engine(Params.builtin(*fixture_tags(g)),
                 dict(zip(L.OPTION_NAMES, [int(x) for x in g["options"]])), device=0, precision=4)
    st, isn, dg, status = run_single(eng, g)
    for c in cols:
        print(f"column {c}: isnow {g['isnow0'][c]} -> {isn[c]} (ref {g['isnow1'][c]}), status {status[c]}")
        for lab, got, ref in (("state", st, g["state1"]), ("diag", dg, g["diag"])):
            names = STATE_NAMES if lab == "state" else L.DIAG_FULL
            for k, nm in enumerate(names):
                a, b = got[k, c], ref[k, c]
                same = a.view(np.int32) == b.view(np.int32) or (np.isnan(a) and np.isnan(b))
                print(f"  {'  ' if same else '!!'} {nm:10s} {a!r:>16} {b!r:>16}")
        print("  inputs:", {n: g["state0"][k, c] for k, n in enumerate(STATE_NAMES)
                            if n in ("TV", "TAH", "EAH", "FWET", "CANLIQ", "CANICE", "TG", "SNEQV")})


if __name__ == "__main__":
    main()
