#!/bin/bash
# fp64 change check: the GPU tests (fp64 tolerance tests included), then
# configs #5 and #2 (fp64) and #3 (fp32, must not move).  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-f64}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" "$OUT/pytest.log" | head -20; exit $rc; }
CFG5="--kind global --ncol 1036800 --precision 8 --opt-veg 2 --dt 3600 --out-every 1 --forcing device"
run() {
  local name=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e6,1), 'step_ms', round(d['roofline']['step_ms'],4))"
}
for rep in 1 2; do
  run cfg5_$rep $CFG5
  run cfg2_$rep --kind casenml --ncol 65536 --precision 8
  run cfg3_$rep
done
