#!/bin/bash
# Round 6, the checked-division build: the bench line (driver's window) five
# times on one box, then config #5's whole year (tools/gpu_r06_year.sh).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06u}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
for k in 1 2 3 4 5; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$O/rep_$k.log" 2>&1 || { echo "rep $k failed"; tail -5 "$O/rep_$k.log"; exit 1; }
  python -c "import json; d=[json.loads(l) for l in open('$O/rep_$k.log') if l.startswith('{\"metric')][-1]; r=d['roofline']; print('rep_$k', round(d['value']/1e6,1), 'Mcs/s gpu_step_ms', round(r['step_ms'],4), 'kernel_ms', round(r['kernel_ms'],4))" | tee -a "$O/repeat.txt"
done
TAG=${TAG:-r06u}/year bash tools/gpu_r06_year.sh
