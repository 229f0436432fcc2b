#!/bin/bash
# Round 6, box G: interleaved A/B of variants against the shipped build on
# config #3 (the driver's arguments), 3 rounds: gmbl = expf/logf special
# cases as selects (NMP_GM_BRANCHLESS=1), re-checked after round 5's spill cut.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06g}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
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
  for v in ${VARIANTS:-default gmbl}; do
    run ${v}_$rep $v --steps 20 --warmup 5
  done
done
echo done
