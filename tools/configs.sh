#!/bin/bash
# Bench lines for the BASELINE.json configs other than the headline (#3), per
# GPU, in the default (coherent) column order and in the generator's order.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-configs}; mkdir -p "$OUT"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps ${STEPS:-48} --warmup 4 "$@" > "$OUT/${name}.json" 2> "$OUT/${name}.err"
  local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 "$OUT/${name}.err"; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/${name}.json')); print('$name', round(d['value']/1e6,1), 'Mcs/s step_ms', round(d['roofline']['step_ms'],3), 'hbm', round(d['roofline']['frac'],4))"
}
# config #4 whole: all 4,194,304 CONUS-like columns on one GPU (8 resident forcing slices)
run cfg4_conus_f32_full_lon-snow-type --kind conus --ncol 4194304 --period 8
for o in lon-snow-type as-generated; do
  run cfg2_casenml_f64_$o --kind casenml --ncol 65536 --precision 8 --order $o
  run cfg4_conus_f32_$o --kind conus --ncol 524288 --order $o
  run cfg5_global_f64_veg2_$o --kind global --ncol 1036800 --precision 8 --opt-veg 2 --dt 3600 --out-every 1 --forcing device --order $o
  run cfg5_global_f32_veg2_$o --kind global --ncol 1036800 --opt-veg 2 --dt 3600 --out-every 1 --forcing device --order $o
done
