#!/bin/bash
# Final build: the cap-and-resume split re-measured (the capped kernels lost
# their spills with the new addressing), and the Fortran slot re-timed.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05x}
mkdir -p "$O"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 "$O/$name.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['value']/1e6,1), 'Mcs/s step_ms', round(r['step_ms'],4))" | tee -a "$O/cap_ab.txt"
}
for rep in 1 2; do
  run plain_$rep
  run cap12_$rep --vege-cap 12 --cap-same-stream
  run cap16_$rep --vege-cap 16 --cap-same-stream
  GPU_MAX_HW_QUEUES=8 run q8pipe12_$rep --vege-cap 12
done
timeout -k 10 600 python -u tools/drop_in_timing.py --ncol 1048576 --steps 20 --out "$O/dropin.json" > "$O/dropin.log" 2>&1
rc=$?; echo "dropin rc=$rc"; tail -8 "$O/dropin.log"
