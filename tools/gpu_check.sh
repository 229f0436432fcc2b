#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step is time-limited; a crash/timeout (rc not in {0,1}) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-check}
mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
export PYTHONUNBUFFERED=1

timeout -k 10 ${T_TEST:-420} python -m pytest tests -m gpu -q -rf --durations=10 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; ok $rc || exit $rc

timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 ${T_BENCH:-400} python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.log"; [ $rc -eq 0 ] || exit $rc

if [ "${PROF:-1}" = 1 ]; then
  R=$PWD
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$R/$OUT/prof.log" 2>&1)
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/prof" -name "*stats*" | head
fi
