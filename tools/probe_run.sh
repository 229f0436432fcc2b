#!/bin/bash
# Timing probes (NOT bit-exact builds, never shipped): how much of the step the
# IEEE division sequence and the glibc-exact libm cost.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-probe}; mkdir -p "$OUT"
run() {
  local name=$1 lib=$2; shift 2
  if [ "$lib" = default ]; then
    timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.log" 2>&1
  else
    NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_$lib.so timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.log" 2>&1
  fi
  [ $? -eq 0 ] || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e6,1), 'step_ms', round(d['roofline']['step_ms'],4))"
}
for rep in 1 2; do
  run base_ref_$rep default
  run base_fast_$rep default --math fast
  run nocrdiv_ref_$rep ${PROBE:-nocrdiv}
done
