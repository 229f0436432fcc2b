#!/bin/bash
# Bench lines for the BASELINE.json configs other than the headline (#3), one
# engine-library variant per line (VARIANTS, default: the in-tree build).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-configs}; mkdir -p "$OUT"
run() {  # name variant args...
  local name=$1 v=$2; shift 2
  local lib=""
  [ "$v" != "base" ] && lib="NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_$v.so"
  env $lib timeout -k 10 240 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 3 --period 8 "$@" > "$OUT/${name}_$v.json" 2> "$OUT/${name}_$v.err"
  local rc=$?; [ $rc -eq 0 ] || { echo "$name $v rc=$rc"; tail -3 "$OUT/${name}_$v.err"; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/${name}_$v.json')); print('$name', '$v', round(d['value']/1e6,1), 'Mcs/s kernel_ms', round(d['roofline']['kernel_ms'],3), 'hbm', round(d['roofline']['frac'],4))"
}
for v in ${VARIANTS:-base}; do
  run cfg5_global_f64_veg2 $v --kind global --ncol 1036800 --precision 8 --opt-veg 2 --dt 3600 --out-every 1
  run cfg2_casenml_f64 $v --kind casenml --ncol 65536 --precision 8 --streams 1
done
for v in ${VARIANTS32:-base}; do
  run cfg4_conus_f32 $v --kind conus --ncol 524288
  run cfg5_global_f32_veg2 $v --kind global --ncol 1036800 --opt-veg 2 --dt 3600 --out-every 1
done
