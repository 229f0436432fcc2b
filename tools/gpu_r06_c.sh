#!/bin/bash
# Round 6, box C: the new GPU tests (config #5 shard pipeline, LDASIN-block
# driver), the N = 8 launch rehearsal (tools/dist_rehearsal8.sh) and the
# per-phase counters (tools/phase_counters.sh on lib_trunc.so).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06c}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "config5_shard or ldasin or netcdf" > "$O/pytest_new.log" 2>&1
rc=$?; tail -3 "$O/pytest_new.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
TAG=${TAG:-r06c}/dist8 bash tools/dist_rehearsal8.sh > "$O/dist8.txt" 2>&1
rc=$?; cat "$O/dist8.txt"; [ $rc -eq 0 ] || { echo "rehearsal rc=$rc"; exit $rc; }
timeout -k 10 600 python -u tools/offline_timing.py --out "$O/offline_driver.json" \
  > "$O/offline_timing.log" 2>&1 || { echo "offline timing failed"; tail -8 "$O/offline_timing.log"; exit 1; }
grep '^{' "$O/offline_timing.log"
MARKS="3 4 5 6 14 9 10 11 13 99" TAG=${TAG:-r06c}/phase bash tools/phase_counters.sh || exit 1
cd "$R" && python tools/phase_counters.py "$O/phase" --out "$O/phase_counters.json"
echo done
