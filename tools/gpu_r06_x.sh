#!/bin/bash
# Round 6, final build: the host paths re-timed at 1,048,576 columns -- the
# Python offline driver in every upload mode (tools/offline_timing.py) and the
# Fortran engine slot (tools/drop_in_timing.py).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06x}
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
step offline 600 python -u tools/offline_timing.py --out "$O/offline_driver.json"
step dropin 500 python -u tools/drop_in_timing.py --ncol 1048576 --steps 20 --out "$O/dropin.json"
echo done
