#!/bin/bash
# Round 6, box I: device COSZ and the once-per-file LDASIN upload
# (nmp_forcing_from_ldasin_geo): its forcing and driver tests, then the offline
# driver timed at 1,048,576 columns in every upload mode (tools/offline_timing.py).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06y}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$O/steps.txt"
  tail -3 "$O/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
step pytest_forcing 300 python -u -m pytest tests/test_gpu_forcing.py tests/test_gpu_driver.py \
  -m gpu -v -s --timeout 240 --timeout-method thread
step offline 600 python -u tools/offline_timing.py --out "$O/offline_driver.json"
echo done
