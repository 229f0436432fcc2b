#!/bin/bash
# Config #3 as the 8-GPU SCALE run holds it: each rank's own 1,048,576-column
# set (seed 1000 + rank) stepped alone on one GPU (--emulate-rank R), the
# driver's window; the slowest rank sets the job's time.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06emul3}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --emulate-rank $r > "$O/r$r.log" 2>&1 || { echo "r$r rc=$?"; tail -3 "$O/r$r.log"; exit 1; }
  python -c "import json; d=[json.loads(l) for l in open('$O/r$r.log') if l.startswith('{\"metric')][-1]; print('rank $r', round(d['value']/1e6,1), 'Mcs/s', round(d['ms_per_step'],4), 'ms/step')" | tee -a "$O/summary.txt"
done
echo done
