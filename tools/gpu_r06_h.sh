#!/bin/bash
# Round 6, box H: the Fortran engine slot's LDASIN-block upload.  Its parity
# tests (bit-exact vs the reference trajectory, and runl == run on the
# host-formed forcing), then the slot timed at 1,048,576 columns with the 12
# forcing fields uploaded vs the 9-field LDASIN block (tools/drop_in_timing.py).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06h}
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
step pytest_slot 300 python -u -m pytest tests/test_gpu_routines.py -m gpu -v -k fortran \
  --timeout 240 --timeout-method thread
step dropin 600 python -u tools/drop_in_timing.py --ncol 1048576 --steps 20 --out "$O/dropin.json"
echo done
