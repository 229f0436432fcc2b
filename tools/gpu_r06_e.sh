#!/bin/bash
# Round 6 closing evidence pass on the final build: the whole GPU suite and
# smoke, the PMC passes of the shipped kernel (HBM bytes, VALU classes, lane
# utilisation: tools/pmc_run.sh -> tools/pmc_traffic.py), the rocprofv3
# kernel statistics of the driver-style bench, the default bench line (with
# the CPU baseline), and the other BASELINE configs (tools/configs.sh).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06e}
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
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_all 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  step bench_driver 300 python -u bench.py --steps 20 --warmup 5
  TAG=${TAG:-r06e}/pmc step pmc 900 bash tools/pmc_run.sh
  step traffic 60 python tools/pmc_traffic.py "$O/pmc" --out "$O/traffic.json"
fi
cd /tmp && export TMPDIR=/tmp
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
cd "$R"
TR=()
[ -f "$O/traffic.json" ] && TR=(--traffic "$O/traffic.json")  # this build's PMC passes
step bench_with_traffic 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "${TR[@]}"
step bench_48 300 python -u bench.py "${TR[@]}"
if [ "${CONFIGS:-1}" = 1 ]; then
  TAG=${TAG:-r06e}/configs step configs 900 bash tools/configs.sh
fi
echo done
