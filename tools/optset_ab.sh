#!/bin/bash
# A/B: compiled option-set kernels vs the run-time-options kernel (NMP_GENERIC_OPTIONS=1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-optset}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" "$OUT/pytest.log" | head; exit $rc; }
run() {
  local name=$1; shift
  timeout -k 10 200 "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e6,1), 'step_ms', round(d['roofline']['step_ms'],4))"
}
for g in 0 1 0 1; do
  run cfg3_g$g env NMP_GENERIC_OPTIONS=$g python bench.py --no-cpu-baseline
  run cfg5_g$g env NMP_GENERIC_OPTIONS=$g python bench.py --no-cpu-baseline --kind global --ncol 1036800 --precision 8 --opt-veg 2 --dt 3600 --out-every 1 --forcing device
done
run cfg2_g0 env NMP_GENERIC_OPTIONS=0 python bench.py --no-cpu-baseline --kind casenml --ncol 65536 --precision 8
run cfg4_g0 env NMP_GENERIC_OPTIONS=0 python bench.py --no-cpu-baseline --kind conus --ncol 524288
