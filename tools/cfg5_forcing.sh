#!/bin/bash
# Config #5 shape on one GPU (1,036,800 global-grid columns, fp64, carbon on,
# output every step): resident forcing slices vs forcing generated on device.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-cfg5}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_forcing.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for fc in resident device resident device; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --kind global --ncol 1036800 --precision 8 --opt-veg 2 --out-every 1 --steps 240 --warmup 4 --forcing $fc > "$OUT/b_$fc.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $fc rc=$rc"; tail -3 "$OUT/b_$fc.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$OUT/b_$fc.log').read().strip().splitlines()[-1]); print('$fc', round(d['value']/1e6,1), 'Mcs/s step_ms', round(d['roofline']['step_ms'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],4))"
done
