#!/bin/bash
# Closing evidence for the shipped build (after the GPU suite has passed on
# it): smoke, the PMC passes, the rocprofv3 kernel statistics of the
# driver-style bench, the driver-style bench line, and the other configs.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05s}
mkdir -p "$O"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$O/steps.txt"
  tail -3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAG=${TAG:-r05s}/pmc step pmc 600 bash tools/pmc_run.sh
cd /tmp && export TMPDIR=/tmp
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
cd "$R"
step bench 200 python -u bench.py --steps 20 --warmup 5
TAG=${TAG:-r05s}/configs step configs 900 bash tools/configs.sh
echo done
