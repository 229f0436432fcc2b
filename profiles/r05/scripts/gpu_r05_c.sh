#!/bin/bash
# Round 5 combined GPU pass.  Each step has its own time limit; a failing test
# or bench (rc 1/2) is recorded and the pass goes on, a timeout, abort or
# crash (rc 124/134/137/139 or > 128) ends it.
#   1 the new GPU tests (cap and resume, mid-loop fallback probe, RCCL gather,
#     exhaustive sqrt, division edges, Fortran slot fp32/fp64)
#   2 cap and resume A/B on config #3 (interleaved, 2 rounds)
#   3 the Fortran slot timed at 1 M columns
#   4 fp64 Estrin exp: accuracy, fp64 tests on the variant, A/B configs #2/#5
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05c}
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
step pytest_new 500 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread \
  -k "vege_cap or midloop or rccl or exhaustive or region_edges or engine_slot or single_call_bit_exact"
for rep in 1 2; do
  for k in 0 12 8 10; do
    step cap${k}_$rep 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --vege-cap $k
    python -c "import json; d=json.loads(open('$O/cap${k}_$rep.log').read().strip().splitlines()[-1]); print('cap $k rep $rep', round(d['value']/1e6,1), 'Mcs/s step_ms', round(d['roofline']['step_ms'],4))" 2>/dev/null | tee -a "$O/cap_ab.txt"
  done
done
step dropin 300 python -u tools/drop_in_timing.py --ncol 1048576 --steps 20 --out "$O/dropin.json"
step exp_estrin 60 tools/exp_estrin_check
NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_f64estrin.so step pytest_f64estrin 300 \
  python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "fp64 or config2"
TAG=${TAG:-r05c}/vab VARIANTS="f64estrin" CFGS="2 5" REPS=2 step f64_ab 600 bash tools/variant_ab.sh
echo done
