#!/bin/bash
# Round 5: stream-range phase offset (unequal ranges) with and without the
# canopy-loop cap, and the config #4 shard's column order (band width).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05f}
mkdir -p "$O"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 "$O/$name.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['value']/1e6,1), 'Mcs/s step_ms', round(r['step_ms'],4), 'range_ms', round(r['kernel_ms'],4))" | tee -a "$O/summary.txt"
}
for rep in 1 2; do
  run split50_$rep
  run split40_$rep --first-range 0.4
  run split30_$rep --first-range 0.3
  run cap12_split40_$rep --vege-cap 12 --first-range 0.4
  run cap12_split30_$rep --vege-cap 12 --first-range 0.3
done
run cap14_split30 --vege-cap 14 --first-range 0.3
for b in 4 8 16; do
  run cfg4_shard_band$b --kind conus --ncol 524288 --order-band $b
done
run cfg4_shard_split30 --kind conus --ncol 524288 --first-range 0.3
echo done
