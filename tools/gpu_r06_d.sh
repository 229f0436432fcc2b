#!/bin/bash
# Round 6, box D: the whole GPU suite on the build with the soil-water short
# division (NMP_SOIL_DIV), then an interleaved A/B against the same sources
# built with NMP_SOIL_DIV=0 (lib_soildiv0.so): config #3 with the driver's
# arguments and config #5's grid (fp64: unaffected, a control), 3 rounds.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06d}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
grep -h "dry clay" "$O/pytest_gpu.log" | head -4
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  if [ "$lib" = default ]; then unset NOAHMP_ENGINE_LIB; else export NOAHMP_ENGINE_LIB="$R/noahmp-1_amd/lib/variants/lib_$lib.so"; fi
  timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  unset NOAHMP_ENGINE_LIB
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 "$O/$name.log"; exit $rc; }
  python -c "import json; d=[json.loads(l) for l in open('$O/$name.log') if l.startswith('{\"metric')][-1]; r=d['roofline']; print('$name', round(d['value']/1e6,1), 'Mcs/s gpu_step_ms', round(r['step_ms'],4))" | tee -a "$O/ab.txt"
}
for rep in 1 2 3; do
  run soil_on_$rep default --steps 20 --warmup 5
  run soil_off_$rep soildiv0 --steps 20 --warmup 5
done
for rep in 1 2; do
  run soil_on_48_$rep default
  run soil_off_48_$rep soildiv0
done
echo done
