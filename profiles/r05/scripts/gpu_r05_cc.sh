#!/bin/bash
# Final build: stream-range count sweep on config #3 (4 and 8 hardware
# queues), and config #5's whole hourly year (8,760 steps, forcing generated
# on the device) in fp64 and fp32.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05cc}
mkdir -p "$O"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 "$O/$name.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['value']/1e6,1), 'Mcs/s ms_per_step', round(d['ms_per_step'],4), 'wall_s', round(d['ms_per_step']*d['steps']/1e3,2))" | tee -a "$O/summary.txt"
}
for rep in 1 2; do
  for s in 1 2 3 4; do run s${s}_$rep --streams $s; done
  GPU_MAX_HW_QUEUES=8 run q8s3_$rep --streams 3
  GPU_MAX_HW_QUEUES=8 run q8s4_$rep --streams 4
done
C5="--kind global --ncol 1036800 --opt-veg 2 --dt 3600 --out-every 1 --forcing device --warmup 24"
run year_f64 $C5 --precision 8 --steps 8760
run year_f32 $C5 --steps 8760
