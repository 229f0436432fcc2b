"""Turn rocprofv3 PMC CSVs (tools/pmc_run.sh) into profiles/traffic.json.

HBM bytes per engine launch = FETCH_SIZE * read-correction + WRITE_SIZE *
write-correction, where the corrections come from the calibration copy
(tools/calib_copy.hip: same SoA 4 B/lane pattern, known byte counts), per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section: FETCH_SIZE is
uncalibrated for non-16B accesses; calibrate on your own pattern).
FETCH_SIZE/WRITE_SIZE are reported in KB (1024 B) by rocprofv3.

usage: python tools/pmc_traffic.py gpurun_out/<tag> [--ncol N] [--streams S] [--out FILE]
(S = the bench's --streams: each dispatch covers ncol/S columns)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "sflx_step_kernel"


def counters(d, counter):
    """{dispatch_id: (kernel_name, value)} from a counter_collection.csv under d."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert files, f"no counter_collection.csv under {d}"
    out = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                r = {k.lower(): v for k, v in row.items()}
                if r.get("counter_name") != counter:
                    continue
                did = r.get("dispatch_id") or r.get("correlation_id")
                name = r.get("kernel_name", "")
                v = float(r["counter_value"])
                k0 = out.get(did, (name, 0.0))
                out[did] = (name, k0[1] + v)  # sum over dimension instances
    return out


def mean_for(d, counter, pat):
    vals = [v for (n, v) in counters(d, counter).values() if pat in n]
    assert vals, (d, counter, pat)
    return sum(vals) / len(vals), len(vals)


def main():
    base = sys.argv[1]
    ncol = 1 << 20
    if "--ncol" in sys.argv:
        ncol = int(sys.argv[sys.argv.index("--ncol") + 1])
    streams = 2
    if "--streams" in sys.argv:
        streams = int(sys.argv[sys.argv.index("--streams") + 1])
    out_every = 6
    if "--out-every" in sys.argv:
        out_every = int(sys.argv[sys.argv.index("--out-every") + 1])
    kind = "mixed"
    if "--kind" in sys.argv:
        kind = sys.argv[sys.argv.index("--kind") + 1]
    order = "lon-snow-type"
    if "--order" in sys.argv:
        order = sys.argv[sys.argv.index("--order") + 1]
    cols_per_launch = ncol / streams
    calib_n, nf = 4194304, 56
    cal_bytes = nf * calib_n * 4
    cf, _ = mean_for(os.path.join(base, "calib_FETCH_SIZE"), "FETCH_SIZE", "calib_soa_copy")
    cw, _ = mean_for(os.path.join(base, "calib_WRITE_SIZE"), "WRITE_SIZE", "calib_soa_copy")
    rf = cal_bytes / (cf * 1024.0)
    rw = cal_bytes / (cw * 1024.0)
    bf, nb = mean_for(os.path.join(base, "bench_FETCH_SIZE"), "FETCH_SIZE", KERNEL)
    bw, _ = mean_for(os.path.join(base, "bench_WRITE_SIZE"), "WRITE_SIZE", KERNEL)
    rd = bf * 1024.0 * rf
    wr = bw * 1024.0 * rw
    sys.path.insert(0, ROOT)
    import noahmp_pkg  # noqa: F401
    from noahmp_amd import build
    # the hash of the library the PMC passes actually measured (the bench line's
    # checks.build_hash), else the sources here
    measured = None
    for lg in glob.glob(os.path.join(base, "bench_*.log")):
        for ln in open(lg, errors="replace"):
            if ln.startswith("{") and '"build_hash"' in ln:
                measured = json.loads(ln)["checks"]["build_hash"]
    res = {"source_hash": measured or build.source_hash(), "ncol": ncol, "streams": streams, "kind": kind,
           "out_every": out_every, "order": order,
           "precision": 4, "math": "ref", "kernel": KERNEL, "dispatches": nb,
           "fetch_size_kb": bf, "write_size_kb": bw, "read_correction": rf,
           "write_correction": rw, "read_bytes": rd, "write_bytes": wr,
           "bytes_per_launch": rd + wr, "bytes_per_colstep": (rd + wr) / cols_per_launch,
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({base})"}
    for sub, names in (("bench_SQ", ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_INSTS_SALU",
                                      "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                                      "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU_INT32",
                                      "SQ_INSTS_VALU_TRANS_F64")),
                       ("bench_SQ2", ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
                                      "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32",
                                      "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                      "SQ_INSTS_VALU_FMA_F64"))):
        sq = os.path.join(base, sub)
        if not os.path.isdir(sq):
            continue
        for c in names:
            try:
                res[c] = mean_for(sq, c, KERNEL)[0]  # per dispatch
            except AssertionError:
                pass
    sq3 = os.path.join(base, "bench_SQ3")
    if os.path.isdir(sq3):
        # VALU lane utilisation (rocprofiler's VALUUtilization expression,
        # counter_defs.yaml: THREAD_CYCLES_VALU / (ACTIVE_INST_VALU x 64)), both
        # counters from the same pass and dispatches
        v = {c: mean_for(sq3, c, KERNEL)[0] for c in
             ("SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_WAVES",
              "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
        res["lane_pass"] = v
        res["lane_util"] = v["SQ_THREAD_CYCLES_VALU"] / (64.0 * v["SQ_ACTIVE_INST_VALU"])
    out = os.path.join(ROOT, "profiles", "traffic.json")
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
