#!/bin/bash
# Round 5 evidence pass: the whole GPU suite, the PMC passes (HBM bytes, VALU
# classes, lane utilisation) of the shipped kernel, the energy-phase probe's
# lane utilisation, the rocprofv3 kernel statistics of the driver-style bench,
# and a kernel trace of the bench with the canopy loop capped at 12 (main vs
# resume launch).  Steps as in gpu_r05_c.sh.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05d}
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
step pytest_all 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAG=${TAG:-r05d}/pmc step pmc 600 bash tools/pmc_run.sh
cd /tmp && export TMPDIR=/tmp
NOAHMP_ENGINE_LIB=$R/noahmp-1_amd/lib/variants/lib_en_w4.so step energy_SQ3 200 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$R/$O/pmc/energy_SQ3" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/ktrace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
step ktrace_cap12 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/ktrace_cap12" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --vege-cap 12
cd "$R"
step bench 200 python -u bench.py --steps 20 --warmup 5
echo done
