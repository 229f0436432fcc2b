#!/bin/bash
# Round 5 second evidence pass: lane utilisation of the energy-phase probe and
# of config #2 (fp64, one wave per SIMD), rocprofv3 kernel statistics of the
# driver-style bench (plain and with the canopy loop capped at 12), the
# pipelined Fortran slot timed at 1 M columns, the division-edge tests, then
# the launch-size study.  Steps as in gpu_r05_c.sh (absolute output paths).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05e}
mkdir -p "$O/pmc"
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
step pytest_edges 300 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread -k "region_edges or engine_slot"
step dropin 400 python -u tools/drop_in_timing.py --ncol 1048576 --steps 20 --out "$O/dropin.json"
SQ3="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
cd /tmp && export TMPDIR=/tmp
NOAHMP_ENGINE_LIB=$R/noahmp-1_amd/lib/variants/lib_en_w4.so step energy_SQ3 200 rocprofv3 --pmc $SQ3 --kernel-trace --output-format csv -d "$O/pmc/energy_SQ3" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline
step cfg2_SQ3 200 rocprofv3 --pmc $SQ3 --kernel-trace --output-format csv -d "$O/pmc/cfg2_SQ3" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --kind casenml --ncol 65536 --precision 8
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
step ktrace_cap12 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace_cap12" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --vege-cap 12
cd "$R"
TAG=${TAG:-r05e}/launch STEPS=20 step launch_study 900 bash tools/launch_study.sh
echo done
