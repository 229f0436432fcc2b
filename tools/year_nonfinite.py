"""Diagnostic (GPU box): the fp32 config #5 year (tools/year_run.sh) ends with
non-finite STC somewhere.  Steps the same column set (global grid, bench seed,
coherent order, opt_veg 2, device forcing, dt 3600, julian wrapped at the
year) in chunks of 48 hourly steps through nmp_run, finds the first chunk
after which STC is non-finite, and re-runs the columns that turned bad from
that chunk's start state with the same forcing slices through the fp32 C
restatement (oracle, the checker only): if it makes the same bits, the
non-finite values are the reference's own.
python tools/year_nonfinite.py [ncol]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from golden_io import bit_equal, load_params  # noqa: E402

import port  # noqa: E402  (oracle: the checker only)


def main():
    from noahmp_amd import cases, layout as L
    from noahmp_amd.engine import ColumnState, Engine
    from noahmp_amd.order import coherent_order
    from noahmp_amd.params import Params
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1036800
    dev, dt, yl, seed, chunk = "cuda:0", 3600.0, 366, 1000, 48
    P = Params.builtin("STAS", "USGS")
    pd = P.as_dict()
    opts = dict(L.CASE_NML_OPTIONS, opt_veg=2)
    otuple = tuple(opts[k] for k in L.OPTION_NAMES)
    cols = cases.make_columns(n, "global", pd, seed=seed, julian=180.0)
    cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, "lon-snow-type"))
    eng = Engine(P, opts, device=0, precision=4)
    cs = ColumnState.from_host(cols, dev)
    st_init, isn_init = cols.state.copy(), cols.isnow.copy()
    clim = torch.as_tensor(cases.climate(cols), device=dev).float().contiguous()
    F = torch.empty((chunk, L.NFORCING, n), device=dev)
    vt = cols.static_i[L.STATIC_I.index("VEGTYP")]
    stc = L.s("STC")
    for c in range(8784 // chunk):
        jul0 = (180.0 + c * chunk * dt / 86400.0) % yl
        for s in range(chunk):
            jul = float(np.float32(jul0) + np.float32(s) * np.float32(dt) / np.float32(86400.0))
            eng.forcing_synth(clim, jul, yl, seed, c * chunk + s, F[s])
        st0, isn0 = cs.state.cpu().numpy().copy(), cs.isnow.cpu().numpy().copy()
        eng.run(cs, F, cases.CASE_NML_ZSOIL, dt, jul0, yl, chunk)
        torch.cuda.synchronize()
        bad = ~torch.isfinite(cs.state[stc]).all(0)
        nb = int(bad.sum())
        if nb == 0:
            continue
        idx = np.nonzero(bad.cpu().numpy())[0]
        print(f"chunk {c} (steps {c * chunk}..{c * chunk + chunk - 1}, julian0 {jul0}): "
              f"{nb} columns with non-finite STC", flush=True)
        sel = idx[:64]
        Fh = F[:, :, torch.as_tensor(sel, device=dev)].cpu().numpy()
        est, eisn, _, estat = port.run(load_params(), otuple, cases.CASE_NML_ZSOIL, dt, yl,
                                       np.float32(jul0), st0[:, sel], isn0[sel],
                                       cols.static_f[:, sel], cols.static_i[:, sel], Fh, chunk)
        got = cs.state.cpu().numpy()[:, sel]
        same = bit_equal(got, est).all(0)
        print(f"  oracle from the chunk start, same forcing: {int(same.sum())}/{sel.size} "
              f"columns bit-identical; oracle non-finite STC in "
              f"{int((~np.isfinite(est[stc])).any(0).sum())}/{sel.size}")
        print("  VEGTYP", np.unique(vt[sel]).tolist(), "SOILTYP",
              np.unique(cols.static_i[L.STATIC_I.index("SOILTYP")][sel]).tolist(),
              "ISNOW at start", np.unique(isn0[sel]).tolist())
        lat = cols.static_f[L.STATIC_F.index("LAT")][sel] if "LAT" in L.STATIC_F else None
        if lat is not None:
            print("  LAT deg", np.round(np.degrees(lat[:8]), 1).tolist())
        c0 = sel[0]
        for nm in ("TV", "TG", "TAH", "SNEQV", "SNOWH", "CANLIQ", "CANICE", "STC", "SH2O"):
            sl = L.s(nm)
            print(f"  col {c0} {nm}: start {st0[sl, c0].tolist()} gpu {got[sl, 0].tolist()}")
        # the reference itself (oracle/_ref), stepped from the year's initial
        # state with the same forcing slices (regenerated: the generator is
        # stateless): where its first non-finite state value appears, and
        # whether its state after chunk c equals the GPU's bit for bit
        import ref
        ref.configure(otuple)
        st, isn = st_init[:, sel].copy(), isn_init[sel].copy()
        first = None
        Fs = torch.empty((L.NFORCING, n), device=dev)
        for cc in range(c + 1):
            j0 = (180.0 + cc * chunk * dt / 86400.0) % yl
            for s in range(chunk):
                k = cc * chunk + s
                jul = float(np.float32(j0) + np.float32(s) * np.float32(dt) / np.float32(86400.0))
                eng.forcing_synth(clim, jul, yl, seed, k, Fs)
                fsel = Fs[:, torch.as_tensor(sel, device=dev)].cpu().numpy()
                st, isn, dg, stat = ref.step(cases.CASE_NML_ZSOIL, dt, yl, jul, st, isn,
                                             cols.static_f[:, sel], cols.static_i[:, sel], fsel)
                nf = ~np.isfinite(st[:, 0])
                if first is None and nf.any():
                    names = [nm for nm in L.STATE_OFF if nf[L.s(nm)].any()]
                    first = k
                    print(f"  reference: first non-finite state at step {k} (julian {jul:.4f}): "
                          f"{names}; status {int(stat[0])}")
                    print("  forcing at that step", np.round(fsel[:, 0], 4).tolist())
        same = bit_equal(got, st).all(0)
        print(f"  reference after chunk {c}: {int(same.sum())}/{sel.size} columns bit-identical "
              f"to the GPU")
        return 0
    print("no non-finite STC over the year")
    return 0


if __name__ == "__main__":
    sys.exit(main())
