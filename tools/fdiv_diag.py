"""Diagnostic (GPU box): every single-call golden fixture through the engine
library named by NOAHMP_ENGINE_LIB (default: the shipped one), reporting per
fixture the columns that are not bit-identical to the reference and the
canopy-loop re-run count (nmp_div_redo_count)."""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import conftest  # noqa: E402,F401  (package alias)
import numpy as np  # noqa: E402
from golden_io import as_ref_status, bit_equal, fixture_tags, load, single_names  # noqa: E402
from noahmp_amd import lib as _l  # noqa: E402
from test_gpu_parity import run_single  # noqa: E402


def main():
    from noahmp_amd.engine import Engine
    from noahmp_amd.params import Params
    from noahmp_amd import layout as L
    lib = _l.load()
    names = sys.argv[1:] or single_names()
    for name in names:
        g = load(f"single_{name}.npz")
        tags = fixture_tags(g)
        eng = Engine(Params.builtin(*tags), dict(zip(L.OPTION_NAMES, [int(x) for x in g["options"]])),
                     device=0, precision=4)
        v = C.c_ulonglong(0)
        lib.nmp_div_redo_count(C.byref(v), 1)
        st, isn, dg, status = run_single(eng, g)
        lib.nmp_div_redo_count(C.byref(v), 1)
        exact = bit_equal(st, g["state1"]).all(0) & bit_equal(dg, g["diag"]).all(0) & \
            (isn == g["isnow1"]) & (as_ref_status(status) == g["status"])
        bad = np.nonzero(~exact)[0]
        print(f"{name:16s} opt_set={eng.option_set()} redo={v.value:5d} "
              f"bad={len(bad)} {bad[:10].tolist()}", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
