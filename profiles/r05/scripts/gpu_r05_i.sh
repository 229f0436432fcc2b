#!/bin/bash
# Round 5 closing evidence for the shipped build: the whole GPU suite, smoke,
# the PMC passes (HBM bytes, VALU classes, lane utilisation), the rocprofv3
# kernel statistics of the driver-style bench, and the driver-style bench line.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05i}
mkdir -p "$O"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$O/steps.txt"
  tail -3 "$O/$name.log"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
  return 0
}
step pytest_all 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAG=${TAG:-r05i}/pmc step pmc 600 bash tools/pmc_run.sh
cd /tmp && export TMPDIR=/tmp
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
cd "$R"
step bench 200 python -u bench.py --steps 20 --warmup 5
echo done
