"""Localise the fp64 wrong results of a library variant (VERDICT r2 item 1:
the fp64 kernels built with -mllvm -disable-machine-cse return NaN states).

    python tools/mcse_probe.py run OUT.npz      # steps with $NOAHMP_ENGINE_LIB (or the default lib)
    python tools/mcse_probe.py cmp A.npz B.npz  # field-by-field / column-by-column report

`run` steps 120,001 mixed columns (the failing test's set) in fp64 with the
compiled option set 1 and with the run-time-options kernel (set 0), one step
with all 58 outputs, then 3 more, and saves state / outputs / statuses.
`cmp` lists, per state field and per output, how many columns differ bitwise
(NaN == NaN), and the first differing columns with their static inputs.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L  # noqa: E402

N = 120_001
STATE_NAMES = [f"{n}[{k}]" if w > 1 else n for n, w in L.STATE_FIELDS for k in range(w)]


def run(out, n=N, precision=8, opt_veg=1):
    import torch
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.params import Params
    dev = "cuda:0"
    dtype = torch.float64 if precision == 8 else torch.float32
    tab = Params.builtin()
    opts = dict(L.CASE_NML_OPTIONS, opt_veg=opt_veg)
    cols = cases.make_columns(n, "mixed", tab.as_dict(), seed=11, julian=170.0)
    F = [torch.as_tensor(cases.forcing_step(cols, 170.0 + s / 48.0, 365, s, seed=11),
                         device=dev).to(dtype) for s in range(4)]
    res = {"static_f": cols.static_f, "static_i": cols.static_i, "isnow0": cols.isnow,
           "cosz": F[0][L.FORCING.index("COSZ")].cpu().numpy()}
    for os_ in (1, 0):
        eng = Engine(tab, opts, device=0, precision=precision)
        got = eng.option_set(os_)
        assert got == (opt_veg if os_ else 0), got
        cs = ColumnState.from_host(cols, dev, dtype)
        d = torch.zeros((L.NDIAG_FULL, n), dtype=dtype, device=dev)
        for s in range(4):
            eng.step(cs, F[s], cases.CASE_NML_ZSOIL, 1800.0, 170.0 + s / 48.0, 365,
                     d if s == 0 else None, L.DIAG_FULL_LEVEL if s == 0 else L.DIAG_NONE)
            torch.cuda.synchronize()
            if s == 0:
                res[f"state1_os{os_}"] = cs.state.cpu().numpy()
                res[f"diag1_os{os_}"] = d.cpu().numpy()
                res[f"status1_os{os_}"] = cs.status.cpu().numpy()
                res[f"isnow1_os{os_}"] = cs.isnow.cpu().numpy()
        res[f"state4_os{os_}"] = cs.state.cpu().numpy()
        res[f"status4_os{os_}"] = cs.status.cpu().numpy()
        eng.close()
    np.savez(out, **res)
    print("saved", out, flush=True)


def dump(out, cols=(0, 1, 2, 10), n=N, precision=8):
    """Values of the NMP_DEBUG_DUMP checkpoints (sflx_kernel.hip NMP_DBG) for a
    few columns, one step of option set 1, from a -DNMP_DEBUG_DUMP library."""
    import ctypes as C
    import torch
    from noahmp_amd import lib as _lib
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.params import Params
    L_ = _lib.load()
    L_.nmp_debug_dump.argtypes = [C.c_longlong, C.c_void_p]
    dev = "cuda:0"
    dtype = torch.float64 if precision == 8 else torch.float32
    tab = Params.builtin()
    cols_ = cases.make_columns(n, "mixed", tab.as_dict(), seed=11, julian=170.0)
    F = torch.as_tensor(cases.forcing_step(cols_, 170.0, 365, 0, seed=11), device=dev).to(dtype)
    eng = Engine(tab, dict(L.CASE_NML_OPTIONS), device=0, precision=precision)
    assert eng.option_set() == 1
    res = {}
    buf = np.zeros(256)
    for c in cols:
        cs = ColumnState.from_host(cols_, dev, dtype)
        assert L_.nmp_debug_dump(int(c), None) == 0
        eng.step(cs, F, cases.CASE_NML_ZSOIL, 1800.0, 170.0, 365)
        torch.cuda.synchronize()
        assert L_.nmp_debug_dump(-1, buf.ctypes.data) == 0
        res[f"c{c}"] = buf.copy()
    eng.close()
    np.savez(out, **res)
    print("saved", out, flush=True)


DBG_NAMES = {}
for it in range(4):
    for k, nm in enumerate(["moz", "fm", "fh", "cmv", "chv", "fv", "rahc", "fhg", "rahg", "rb",
                            "estv", "destv", "cah", "cvh", "cgh", "ata", "bta", "caw", "cew",
                            "ctw", "cgw", "aea", "bea", "cev", "ctr", "rssun", "rssha", "tah",
                            "eah", "irc", "shc", "evc", "tr", "dtv", "tv", "h", "hg", "qsfc",
                            "sav", "a"]):
        DBG_NAMES[it * 40 + k] = f"it{it + 1 if it < 3 else 'last'}.{nm}"
for k in range(4):
    for base, nm in ((160, "wdf"), (164, "wcnd"), (168, "ai"), (172, "bi"), (176, "ci"),
                     (180, "rhstt"), (184, "sh2o"), (188, "etrani"), (192, "pp"), (196, "smc")):
        DBG_NAMES[base + k] = f"{nm}[{k}]"
for k, nm in enumerate(["qinfil", "qseva", "qinsrf", "dtfine", "niter", "smcmax", "bexp",
                        "dwsat"]):
    DBG_NAMES[200 + k] = nm
for k, nm in enumerate(["hcan", "zpd", "z0mg", "z0h", "fv", "vai", "cwp", "cwpc", "tmp1", "tmp2",
                        "tmprah2", "kh", "rahg", "tmprb", "fhg", "z0hg"]):
    DBG_NAMES[208 + k] = "ragrb1." + nm


def cmpdump(pa, pb):
    A, B = np.load(pa), np.load(pb)
    for key in A.files:
        a, b = A[key], B[key]
        print(f"== column {key[1:]}")
        for i in range(256):
            if np.isnan(a[i]) and np.isnan(b[i]):
                continue
            flag = "" if a[i] == b[i] else "   <-- differs"
            print(f"  {DBG_NAMES.get(i, i)!s:>14}: {a[i]!r:>24} {b[i]!r:>24}{flag}")


def neq(a, b):
    """Bitwise difference per element (NaN == NaN)."""
    return a.view(np.uint64 if a.dtype == np.float64 else np.uint32) != \
        b.view(np.uint64 if b.dtype == np.float64 else np.uint32)


def cmp(pa, pb):
    A, B = np.load(pa), np.load(pb)
    si, sf = A["static_i"], A["static_f"]
    lines = []
    for key, names in (("state1_os1", STATE_NAMES), ("diag1_os1", L.DIAG_FULL),
                       ("state1_os0", STATE_NAMES), ("diag1_os0", L.DIAG_FULL),
                       ("state4_os1", STATE_NAMES), ("state4_os0", STATE_NAMES)):
        d = neq(A[key], B[key])
        bad = d.any(0)
        lines.append(f"== {key}: {int(bad.sum())} of {bad.size} columns differ; "
                     f"non-finite A {int((~np.isfinite(A[key])).any(0).sum())} "
                     f"B {int((~np.isfinite(B[key])).any(0).sum())}")
        for i in np.argsort(-d.sum(1)):
            if d[i].sum() == 0:
                break
            lines.append(f"   {names[i]:>10s}: {int(d[i].sum())} cols")
        cols = np.nonzero(bad)[0][:12]
        for c in cols:
            f = np.nonzero(d[:, c])[0]
            lines.append(f"   col {c}: vegtyp {si[0, c]} soiltyp {si[1, c]} ist {si[4, c]} "
                         f"isnow0 {A['isnow0'][c]} cosz {A['cosz'][c]:.3f} fields {[names[k] for k in f[:8]]} "
                         f"A {[float(A[key][k, c]) for k in f[:3]]} "
                         f"B {[float(B[key][k, c]) for k in f[:3]]}")
    for key in ("status1_os1", "status1_os0", "status4_os1", "status4_os0", "isnow1_os1"):
        lines.append(f"== {key}: {int((A[key] != B[key]).sum())} differ, nonzero A "
                     f"{int((A[key] != 0).sum())} B {int((B[key] != 0).sum())}")
    # which kernel is wrong: os1 vs os0 within each library
    for tag, Z in (("A", A), ("B", B)):
        lines.append(f"== {tag}: os1 vs os0 state1 differ in "
                     f"{int(neq(Z['state1_os1'], Z['state1_os0']).any(0).sum())} cols, diag1 "
                     f"{int(neq(Z['diag1_os1'], Z['diag1_os0']).any(0).sum())}, state4 "
                     f"{int(neq(Z['state4_os1'], Z['state4_os0']).any(0).sum())}")
    print("\n".join(lines))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], *(int(x) for x in sys.argv[3:]))
    elif sys.argv[1] == "dump":
        dump(sys.argv[2])
    elif sys.argv[1] == "cmpdump":
        cmpdump(sys.argv[2], sys.argv[3])
    else:
        cmp(sys.argv[2], sys.argv[3])
