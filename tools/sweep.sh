#!/bin/bash
# Time engine build variants (noahmp-1_amd/lib/variants/lib_*.so) with bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-sweep}; mkdir -p "$OUT"
for v in ${VARIANTS:-base}; do
  for m in ${MATHS:-ref fast}; do
    NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_$v.so timeout -k 10 180 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup ${WARMUP:-3} --period 8 --math $m ${BENCH_ARGS:-} > "$OUT/${v}_$m.json" 2> "$OUT/${v}_$m.err"
    rc=$?; [ $rc -eq 0 ] || { echo "$v $m rc=$rc"; tail -3 "$OUT/${v}_$m.err"; exit $rc; }
    python -c "import json,sys; d=json.load(open('$OUT/${v}_$m.json')); print('$v', '$m', round(d['value']/1e6,1), 'Mcs/s kernel_ms', round(d['roofline']['kernel_ms'],3))"
  done
done
