#!/bin/bash
# Re-binning sweep on the bench workload (config #3): tile size x re-sort interval.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-rebin}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "rebinned or cost_key" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-"0 1" "256 1" "1024 1" "4096 1" "16384 1" "4096 2" "4096 4"}; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --rebin-tile $1 --rebin-every $2 > "$OUT/bench_$1_$2.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $1 $2 rc=$rc"; tail -3 "$OUT/bench_$1_$2.log"; exit $rc; }
  python - "$OUT/bench_$1_$2.log" $1 $2 <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"tile {sys.argv[2]:>6} every {sys.argv[3]}: {d['value']/1e6:8.1f} Mcs/s  step {d['roofline']['step_ms']:.4f} ms  kernel {d['roofline']['kernel_ms']:.4f} ms")
PY
done
