"""Per-phase counters from the truncation runs of tools/phase_counters.sh.

Mark k = the kernel returns from the column's step when it reaches phase
mark k (csrc/sflx_kernel.hip NMP_PHASE), i.e. it runs every phase before the
mark.  Marks in execution order; consecutive differences are phases:

  2 prelude + first-layer conductivity, 3 radiation, 4 btran + rsurf,
  5 canopy Newton loop (vege_flux), 6 bare-ground loop (bare_flux),
  14 aggregation, 9 thermoprop + tsnosoi + phasechange, 10 canwater,
  11 snowwater, 13 frozen ground + soil water + groundwater,
  99 carbon + balance checks + the rest (no truncation).

Per phase: kernel time (kernel-trace mean per dispatch), VALU
wave-instructions per wave, lane utilisation (SQ_THREAD_CYCLES_VALU / 64
SQ_ACTIVE_INST_VALU), the instruction-class mix (f32 add/mul/fma,
transcendental, f64, int32, other), SALU / branch / LDS / VMEM counts, and the
wait share (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES).

    python tools/phase_counters.py gpurun_out/<tag> [--out profiles/r06/phase_counters.json]
                                   [--label "config #5 fp64"]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "sflx_step_kernel"
ORDER = [2, 3, 4, 5, 6, 14, 9, 10, 11, 13, 99]
NAMES = {2: "prelude + df_top", 3: "radiation", 4: "btran + rsurf", 5: "vege_flux (canopy loop)",
         6: "bare_flux", 14: "aggregation", 9: "thermoprop + tsnosoi + phasechange",
         10: "canwater", 11: "snowwater", 13: "frozen ground + soilh2o + groundwater",
         99: "carbon + checks + rest"}


def counters(d):
    """{counter: mean over the engine kernel's dispatches} of a PMC pass."""
    acc = defaultdict(float)
    seen = defaultdict(set)
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            r = {k.lower(): v for k, v in row.items()}
            if KERNEL not in r.get("kernel_name", ""):
                continue
            c = r["counter_name"]
            acc[c] += float(r["counter_value"])
            seen[c].add(r.get("dispatch_id") or r.get("correlation_id"))
    return {c: v / len(seen[c]) for c, v in acc.items()}


def kernel_ms(d):
    ds = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            r = {k.lower(): v for k, v in row.items()}
            if KERNEL in r.get("kernel_name", ""):
                ds.append((int(r["end_timestamp"]) - int(r["start_timestamp"])) * 1e-6)
    # the bench's steps after the first (warm-up) dispatches: the last 8
    return sum(ds[-8:]) / len(ds[-8:]), len(ds)


def main():
    base = sys.argv[1]
    marks = [k for k in ORDER if os.path.isdir(os.path.join(base, f"m{k}"))]
    cum = {}
    for k in marks:
        d = os.path.join(base, f"m{k}")
        v = {}
        for p in ("p1", "p2", "p3"):
            v.update(counters(os.path.join(d, p)))
        v["kernel_ms"], v["dispatches"] = kernel_ms(os.path.join(d, "kt"))
        cum[k] = v
    phases, prev = [], None
    names = dict(NAMES)
    if marks and marks[0] == 3:  # no mark 2 run: the first row holds the prelude too
        names[3] = "prelude + df_top + radiation"
    for k in marks:
        c = cum[k]
        d = {x: c[x] - (prev[x] if prev else 0.0) for x in c if isinstance(c[x], float)}
        waves = c["SQ_WAVES"]
        f32 = sum(d.get(f"SQ_INSTS_VALU_{o}_F32", 0.0) for o in ("ADD", "MUL", "FMA"))
        f64 = sum(d.get(f"SQ_INSTS_VALU_{o}_F64", 0.0) for o in ("ADD", "MUL", "FMA"))
        tr = d.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
        i32 = d.get("SQ_INSTS_VALU_INT32", 0.0)
        valu = d.get("SQ_INSTS_VALU", 0.0)
        other = valu - f32 - f64 - tr - i32
        # SIMD cycles per wave64 instruction by class (bench.py VALU_CYCLES)
        wcyc = 2 * f32 + 4 * f64 + 8 * tr + 2 * i32 + 2 * other
        ph = {"mark": k, "phase": names.get(k, str(k)),
              "kernel_ms": d["kernel_ms"],
              "valu_per_wave": valu / waves,
              "lane_util": (d["SQ_THREAD_CYCLES_VALU"] / (64.0 * d["SQ_ACTIVE_INST_VALU"])
                            if d.get("SQ_ACTIVE_INST_VALU", 0) > 0 else None),
              "mix_per_wave": {"f32": f32 / waves, "f64": f64 / waves, "trans_f32": tr / waves,
                               "int32": i32 / waves, "other": other / waves},
              "weighted_valu_cycles_per_wave": wcyc / waves,
              "salu_per_wave": d.get("SQ_INSTS_SALU", 0.0) / waves,
              "branch_per_wave": d.get("SQ_INSTS_BRANCH", 0.0) / waves,
              "lds_per_wave": d.get("SQ_INSTS_LDS", 0.0) / waves,
              "vmem_rd_per_wave": d.get("SQ_INSTS_VMEM_RD", 0.0) / waves,
              "vmem_wr_per_wave": d.get("SQ_INSTS_VMEM_WR", 0.0) / waves,
              "wait_inst_share": (d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]
                                  if d.get("SQ_WAVE_CYCLES", 0) > 0 else None),
              "wave_cycles_per_wave": d.get("SQ_WAVE_CYCLES", 0.0) / waves}
        phases.append(ph)
        prev = c
    tot_ms = cum[marks[-1]]["kernel_ms"]
    tot_w = sum(p["weighted_valu_cycles_per_wave"] for p in phases)
    for p in phases:
        p["time_share"] = p["kernel_ms"] / tot_ms
        p["weighted_valu_share"] = p["weighted_valu_cycles_per_wave"] / tot_w
    label = sys.argv[sys.argv.index("--label") + 1] if "--label" in sys.argv else "config #3"
    out = {"source": f"tools/phase_counters.sh truncation runs ({base}); lib_trunc.so "
                     f"(-DNMP_TRUNC_RUNTIME), {label} bench, 4 steps after 1",
           "cumulative": {str(k): cum[k] for k in marks}, "phases": phases}
    print(f"{'phase':42s} {'ms':>7s} {'time%':>6s} {'VALU/wave':>9s} {'lane':>5s} "
          f"{'f32':>6s} {'f64':>6s} {'trans':>6s} {'other':>6s} {'wait%':>6s}")
    for p in phases:
        m = p["mix_per_wave"]
        lu = p["lane_util"]
        wt = p["wait_inst_share"]
        print(f"{p['phase']:42s} {p['kernel_ms']:7.4f} {100 * p['time_share']:6.1f} "
              f"{p['valu_per_wave']:9.0f} {lu if lu is not None else float('nan'):5.2f} "
              f"{m['f32']:6.0f} {m['f64']:6.0f} {m['trans_f32']:6.0f} {m['other']:6.0f} "
              f"{100 * (wt if wt is not None else float('nan')):6.1f}")
    if "--out" in sys.argv:
        path = sys.argv[sys.argv.index("--out") + 1]
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
