#!/bin/bash
# Round 6, final build: config #5 for a whole hourly year (8,760 steps, forcing
# generated on the device, output every step) on one GPU -- the grid in fp64
# and fp32, and each of its eight 129,600-column fp64 shards alone
# (--emulate-rank R), i.e. the compute of the 8-GPU year rank by rank.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06year}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 "$O/$name.log"; exit $rc; }
  python -c "import json; d=[json.loads(l) for l in open('$O/$name.log') if l.startswith('{\"metric')][-1]; print('$name', round(d['value']/1e6,1), 'Mcs/s ms_per_step', round(d['ms_per_step'],4), 'wall_s', round(d['ms_per_step']*d['steps']/1e3,2))" | tee -a "$O/summary.txt"
}
C5="--kind global --opt-veg 2 --dt 3600 --out-every 1 --forcing device --warmup 24"
run year_f64 $C5 --ncol 1036800 --precision 8 --steps 8760
run year_f32 $C5 --ncol 1036800 --steps 8760
for r in 0 1 2 3 4 5 6 7; do
  run year_shard_f64_r$r $C5 --ncol 129600 --precision 8 --steps 8760 --emulate-rank $r
done
echo done
