#!/bin/bash
# Round 5, second GPU pass: the fp64 Estrin exp (accuracy, fp64 tests, A/B on
# configs #2 and #5), lane utilisation (SQ_THREAD_CYCLES_VALU) of the shipped
# kernel and of the energy-phase probe, PMC traffic, and the rocprofv3 kernel
# statistics of the bench.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05b}
mkdir -p "$O"
timeout -k 10 60 tools/exp_estrin_check > "$O/exp_estrin_check.txt" 2>&1
rc=$?; echo "exp check rc=$rc"; cat "$O/exp_estrin_check.txt"; [ $rc -eq 0 ] || exit $rc
NOAHMP_ENGINE_LIB=$R/noahmp-1_amd/lib/variants/lib_f64estrin.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fp64 or config2" > "$O/pytest_f64estrin.log" 2>&1
rc=$?; echo "fp64 tests on the Estrin variant rc=$rc"; tail -2 "$O/pytest_f64estrin.log"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05b}/vab VARIANTS="f64estrin" CFGS="2 5" REPS=2 bash tools/variant_ab.sh
rc=$?; echo "variant A/B rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05b}/cap VARIANTS="cap8 cap10 cap12 cap14" CFGS="3" REPS=2 bash tools/variant_ab.sh
rc=$?; echo "cap probes rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05b}/pmc bash tools/pmc_run.sh
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
NOAHMP_ENGINE_LIB=$R/noahmp-1_amd/lib/variants/lib_en_w4.so timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$R/$O/pmc/energy_SQ3" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$R/$O/pmc/energy_SQ3.log" 2>&1
rc=$?; echo "energy probe SQ3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/ktrace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/ktrace_bench.log" 2>&1
rc=$?; echo "kernel trace rc=$rc"; tail -c 300 "$R/$O/ktrace_bench.log"; exit $rc
