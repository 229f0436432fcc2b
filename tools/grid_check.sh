#!/bin/bash
# Grid sizes of the step kernel's launches (rocprofv3 kernel trace), default
# bench and NMP_RESIDENT=0.  GPU box.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-grid}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for m in 1 0; do
  NMP_RESIDENT=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt$m" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/kt$m.log" 2>&1 || exit 1
  python3 - "$OUT/kt$m/run_kernel_trace.csv" $m <<'PY'
import csv, sys, collections
g = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "sflx_step" in r["Kernel_Name"]:
        g[(r.get("Grid_Size") or r.get("Grid_Size_X"), r.get("Workgroup_Size") or r.get("Workgroup_Size_X"))] += 1
print("NMP_RESIDENT=" + sys.argv[2], dict(g))
PY
done
