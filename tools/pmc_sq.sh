#!/bin/bash
# SQ counters for the engine kernel (one pass, --kernel-trace only):
# VALU issue share, wave stall split.  Usage on the GPU box.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-sq}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"}
timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/sq" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --period 4 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/sq.log" 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/sq.log"; exit $rc; }
python3 - "$OUT/sq/run_counter_collection.csv" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "sflx" in r["Kernel_Name"]:
        acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
tot = collections.defaultdict(float); n = collections.Counter()
for (d, c), v in acc.items():
    tot[c] += sum(v); n[c] += 1
for c in sorted(tot):
    print(f"{c:24s} {tot[c] / n[c]:.4g} per dispatch")
PY
