#!/bin/bash
# Occupancy re-sweep after the option-set kernels (round 2): GPU tests, then the
# default library against waves-per-SIMD variants (tools/build_variants.py
# w3 w5 d3) on config #3 (fp32) and config #5 (fp64, device forcing), then the
# PMC traffic passes and a kernel-trace summary of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-occ}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" "$OUT/pytest.log" | head; exit $rc; }
CFG5="--kind global --ncol 1036800 --precision 8 --opt-veg 2 --dt 3600 --out-every 1 --forcing device"
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
  run cfg3_base_$rep default
  run cfg3_w3_$rep w3
  run cfg3_w5_$rep w5
  run cfg5_base_$rep default $CFG5
  run cfg5_d3_$rep d3 $CFG5
done
[ "${PMC:-1}" = 1 ] || exit 0
TAG=${TAG:-occ}_pmc VALU=1 bash tools/pmc_run.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/ktrace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/ktrace.log" 2>&1
echo "ktrace rc=$?"
