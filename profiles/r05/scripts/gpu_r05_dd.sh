#!/bin/bash
# Round-5 final pass on the shipped build: the whole GPU suite, smoke, the PMC
# passes (profiles/traffic.json), the kernel statistics and the bench lines.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05dd}
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
step pytest_all 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAG=${TAG:-r05dd}/pmc step pmc 600 bash tools/pmc_run.sh
cd /tmp && export TMPDIR=/tmp
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
cd "$R"
echo done
