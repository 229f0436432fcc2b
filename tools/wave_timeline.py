"""How full do the wave slots stay during a step?  (GPU box; variant libraries
built with -DNMP_WAVE_TIMING, tools/build_variants.py wt wt_b128 wt_b64.)

Runs the bench workload (config #3 columns in the coherent order, resident
forcing) for a few steps with S stream ranges, reads every wave's
{start, end} (s_memrealtime, 100 MHz), and reports over the timed steps:

* busy: the integral of resident waves over the window / (wave slots x window)
  -- the slots are 4 waves/SIMD x 4 SIMDs x 256 CUs unless --slots says else;
* wg_idle: for each workgroup, sum over its waves of (last wave's end - this
  wave's end) -- slot time held by a workgroup whose own waves are done (the
  LDS is released per workgroup), as a share of the slot time;
* tail: the time from the last wave start to the last wave end, per launch;
* the spread of wave durations (p10/p50/p90/max).

    python tools/wave_timeline.py [variant=wt] [streams=2] [steps=6] [ncol=1048576]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
variant = sys.argv[1] if len(sys.argv) > 1 else "wt"
os.environ.setdefault("NOAHMP_ENGINE_LIB",
                      os.path.join(ROOT, "noahmp-1_amd", "lib", "variants", f"lib_{variant}.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import cases, layout as L  # noqa: E402
from noahmp_amd.engine import ColumnState, Engine, StreamShards  # noqa: E402
from noahmp_amd.order import coherent_order  # noqa: E402
from noahmp_amd.params import Params  # noqa: E402


def main():
    nstreams = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 20
    slots = 4 * 4 * 256
    P = Params.builtin()
    cols = cases.make_columns(n, "mixed", P.as_dict(), seed=1000, julian=180.0)
    cols = cols.take(coherent_order(cols.lon, cols.static_i, cols.isnow, "lon-snow-type"))
    eng = Engine(P, dict(L.CASE_NML_OPTIONS), 0, 4, "ref")
    lib = eng._lib
    lib.nmp_debug_wave_records.argtypes = [C.c_void_p, C.c_longlong, C.c_int]
    lib.nmp_debug_wave_records.restype = C.c_longlong
    cs = ColumnState.from_host(cols, "cuda:0", torch.float32)
    F = [torch.as_tensor(cases.forcing_step(cols, 180.0 + s / 48.0, 366, s, seed=1000),
                         device="cuda:0").to(torch.float32) for s in range(8)]
    sh = StreamShards(eng, cs, nstreams)
    warm = 3
    for s in range(warm + steps):
        if s == warm:
            sh.join()
            torch.cuda.synchronize()
            lib.nmp_debug_wave_records(None, 0, 1)
        sh.step(F[s % 8], cases.CASE_NML_ZSOIL, 1800.0, 180.0 + s / 48.0, 366)
    sh.join()
    torch.cuda.synchronize()
    cnt = lib.nmp_debug_wave_records(None, 0, 0)
    buf = np.zeros((min(cnt, 1 << 17), 4), dtype=np.uint64)
    got = lib.nmp_debug_wave_records(buf.ctypes.data, buf.shape[0], 1)
    assert got == cnt, (got, cnt)
    if cnt > buf.shape[0]:
        print(f"warning: {cnt} waves, {buf.shape[0]} recorded")
    t0 = buf[:, 0].astype(np.int64)
    t1 = buf[:, 1].astype(np.int64)
    base = t0.min()
    t0 -= base
    t1 -= base
    blk = (buf[:, 3] & np.uint64(0xffffffff)).astype(np.int64)
    tag = (buf[:, 3] >> np.uint64(32)).astype(np.int64)
    dur = t1 - t0
    span = t1.max()
    tick_us = 0.01
    # resident-wave integral over the window
    busy = dur.sum() / (slots * span)
    # workgroup idle: waves of one workgroup share (tag, blk); launches of
    # different steps reuse (tag, blk), so split them by start time as well
    order = np.lexsort((t0, blk, tag))
    key_t = tag[order] * (1 << 24) + blk[order]
    wg_idle = 0
    i = 0
    m = len(order)
    wpb = None
    while i < m:
        j = i + 1
        while j < m and key_t[j] == key_t[i] and t0[order[j]] - t0[order[i]] < 2000:
            j += 1
        e = t1[order[i:j]]
        wg_idle += (e.max() - e).sum()
        wpb = j - i if wpb is None else wpb
        i = j
    # per launch: group by tag, then by step (start-time clusters)
    print(f"variant={variant} streams={nstreams} steps={steps} ncol={n} waves={cnt} "
          f"waves/workgroup={wpb}")
    print(f"window {span * tick_us:.1f} us = {span * tick_us / steps:.1f} us/step; "
          f"busy {100 * busy:.1f} % of {slots} slots; "
          f"wg_idle {100 * wg_idle / (slots * span):.1f} % of slot time "
          f"({100 * wg_idle / dur.sum():.1f} % of wave time)")
    q = np.percentile(dur, [10, 50, 90, 99]) * tick_us
    print(f"wave duration us: p10 {q[0]:.0f} p50 {q[1]:.0f} p90 {q[2]:.0f} p99 {q[3]:.0f} "
          f"max {dur.max() * tick_us:.0f}")
    # resident-wave profile in 20 bins of the window
    edges = np.linspace(0, span, 41)
    prof = []
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(t1, b) - np.maximum(t0, a), 0, None).sum()
        prof.append(ov / ((b - a) * slots))
    print("resident/slots over the window (40 bins): " +
          " ".join(f"{100 * p:.0f}" for p in prof))
    for tg in np.unique(tag):
        sel = tag == tg
        st = np.sort(t0[sel])
        # steps: split where the start times jump by more than half the mean spacing
        gaps = np.where(np.diff(st) > 5000)[0]
        print(f"launch tag {tg:#x}: {sel.sum()} waves, start clusters {len(gaps) + 1}")
    # per step tail (all launches): last start -> last end within each step window
    stp = span / steps
    tails = []
    for k in range(steps):
        sel = (t0 >= k * stp - 0.1 * stp) & (t0 < (k + 1) * stp)
        if sel.sum():
            tails.append((t1[sel].max() - t0[sel].max()) * tick_us)
    print("last-start -> last-end per step window (us): " + " ".join(f"{x:.0f}" for x in tails))


if __name__ == "__main__":
    main()
