#!/bin/bash
# A/B of engine build variants (tools/build_variants.py) against the default
# library, on config #3 (fp32) and config #5 (fp64, device forcing), REPS
# rounds interleaved.  GPU box.  VARIANTS="vu2 pinnv" CFGS="3 5" REPS=2.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-vab}; mkdir -p "$OUT"
CFG5="--kind global --ncol 1036800 --precision 8 --opt-veg 2 --dt 3600 --out-every 1 --forcing device"
CFG2="--kind casenml --ncol 65536 --precision 8"
# a variant "lib@VAR=value" runs library lib with that environment variable set
run() {
  local name=$1 spec=$2; shift 2
  local lib=${spec%%@*} envs=""
  [ "$spec" != "$lib" ] && envs=${spec#*@}
  if [ "$lib" = default ]; then
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.log" 2>&1
  else
    env $envs NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_$lib.so timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.log" 2>&1
  fi
  [ $? -eq 0 ] || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e6,1), 'step_ms', round(d['roofline']['step_ms'],4))"
}
for rep in $(seq 1 ${REPS:-2}); do
  for v in default ${VARIANTS:-}; do
    for c in ${CFGS:-3 5}; do
      if [ "$c" = 5 ]; then run cfg5_${v}_$rep $v $CFG5
      elif [ "$c" = 2 ]; then run cfg2_${v}_$rep $v $CFG2
      else run cfg3_${v}_$rep $v; fi
    done
  done
done
