#!/bin/bash
# Config #5 shape over a whole year of hourly steps (8,784, leap year) on one
# GPU: fp64 and fp32, carbon on, forcing generated on the device, output every
# step.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-year}; mkdir -p "$OUT"
for p in 8 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --kind global --ncol 1036800 --precision $p --opt-veg 2 \
    --dt 3600 --out-every 1 --forcing device --steps 8784 --warmup 4 > "$OUT/year_f$p.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "year fp$p rc=$rc"; tail -3 "$OUT/year_f$p.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$OUT/year_f$p.log').read().strip().splitlines()[-1]); print('fp$p', round(d['value']/1e6,1), 'Mcs/s', round(d['ms_per_step']*d['steps']/1e3,2), 's', d['checks'])"
done
