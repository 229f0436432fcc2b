#!/bin/bash
# Round 6, box B: the GPU tests and smoke on the build without the cap
# experiment and with nmp_forcing_from_ldasin, then tools/gpu_r06_a.sh
# (config #3 + config #5 shards + forced-collective runs) and the offline
# driver at 1,048,576 columns (tools/offline_timing.py).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06b}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -5 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
TAG=${TAG:-r06b}/a bash tools/gpu_r06_a.sh || exit 1
timeout -k 10 600 python -u tools/offline_timing.py --out "$O/offline_driver.json" \
  > "$O/offline_timing.log" 2>&1 || { echo "offline timing failed"; tail -8 "$O/offline_timing.log"; exit 1; }
tail -12 "$O/offline_timing.log"
echo done
