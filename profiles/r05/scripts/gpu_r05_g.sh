#!/bin/bash
# Round 5: staggered stream ranges (with and without the canopy-loop cap),
# 3/4 stream ranges with 8 hardware queues, and wider column-order bands.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05g}
mkdir -p "$O"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 "$O/$name.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['value']/1e6,1), 'Mcs/s step_ms', round(r['step_ms'],4), 'range_ms', round(r['kernel_ms'],4))" | tee -a "$O/summary.txt"
}
for rep in 1 2; do
  run plain_$rep
  run stagger_$rep --stagger
  run cap12_stagger_$rep --vege-cap 12 --stagger
  run cap10_stagger_$rep --vege-cap 10 --stagger
done
GPU_MAX_HW_QUEUES=8 run s4_q8 --streams 4
GPU_MAX_HW_QUEUES=8 run s4_q8_cap12 --streams 4 --vege-cap 12
GPU_MAX_HW_QUEUES=8 run s3_q8_cap12 --streams 3 --vege-cap 12
for b in 8 16; do run band$b --order-band $b; done
run cfg4_shard_band32 --kind conus --ncol 524288 --order-band 32
echo done
