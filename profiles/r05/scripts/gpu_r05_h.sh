#!/bin/bash
# Round 5: the deferred cap-and-resume pipeline -- parity tests, then an
# interleaved A/B on config #3 (2 stream ranges, each with its companion),
# with the default 4 and with 8 hardware queues.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05h}
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread -k "vege_cap or midloop" > "$O/pytest_cap.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/pytest_cap.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() {  # name args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 "$O/$name.log"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['value']/1e6,1), 'Mcs/s step_ms', round(r['step_ms'],4), 'range_ms', round(r['kernel_ms'],4))" | tee -a "$O/summary.txt"
}
for rep in 1 2; do
  run plain_$rep
  run pipe12_$rep --vege-cap 12
  run pipe10_$rep --vege-cap 10
  run pipe14_$rep --vege-cap 14
  GPU_MAX_HW_QUEUES=8 run q8_plain_$rep
  GPU_MAX_HW_QUEUES=8 run q8_pipe12_$rep --vege-cap 12
  GPU_MAX_HW_QUEUES=8 run q8_pipe10_$rep --vege-cap 10
done
echo done
