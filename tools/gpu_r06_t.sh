#!/bin/bash
# Round 6, box T: CTR, TR, DTV and the bare DTG on the short division with
# per-lane numerator windows (NMP_VD_CHECKED, variant lib_vdchk).  1) the GPU
# parity and routine tests on the variant library (bit-exact vs the reference
# fixtures), 2) the fallback rate of the windows (lib_vdchk_fb), 3) interleaved
# A/B on config #3 against the shipped build and the unchecked ceiling
# (AB_ONLY=1: the A/B alone; VARIANTS, REPS).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06t}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
V=$R/noahmp-1_amd/lib/variants
if [ -z "${AB_ONLY:-}" ]; then
NOAHMP_ENGINE_LIB=$V/lib_vdchk.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_routines.py \
  -k "not year" -p no:cacheprovider > "$O/pytest_vdchk.log" 2>&1 || { tail -30 "$O/pytest_vdchk.log"; exit 1; }
tail -2 "$O/pytest_vdchk.log"
NOAHMP_ENGINE_LIB=$V/lib_vdchk_fb.so timeout -k 10 300 python -u tools/fallback_rate.py > "$O/fallback_vdchk.txt" 2>&1 || { tail -20 "$O/fallback_vdchk.txt"; exit 1; }
cat "$O/fallback_vdchk.txt"
fi
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  if [ "$lib" = default ]; then unset NOAHMP_ENGINE_LIB; else export NOAHMP_ENGINE_LIB="$V/lib_$lib.so"; fi
  timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  unset NOAHMP_ENGINE_LIB
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 "$O/$name.log"; exit $rc; }
  python -c "import json; d=[json.loads(l) for l in open('$O/$name.log') if l.startswith('{\"metric')][-1]; r=d['roofline']; print('$name', round(d['value']/1e6,1), 'Mcs/s gpu_step_ms', round(r['step_ms'],4))" | tee -a "$O/ab.txt"
}
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-default vdchk vdchk1 vdallfast}; do
    run ${v}_$rep $v --steps 20 --warmup 5
  done
done
echo done
