#!/bin/bash
# Round 3: guarded fast fp32 division -- parity (incl. the forced re-run
# tests) on the default library, then A/B default (fast + re-run) vs fd2
# (fast, no re-run) vs fd0 (IEEE division everywhere).  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "fast_division or order_check" -s > gpurun_out/fdiv_tests.log 2>&1
rc=$?; echo "fast-division tests rc=$rc"; tail -5 gpurun_out/fdiv_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
TAG=fdivab VARIANTS="fd2 fd0" CFGS="3 5" REPS=2 bash tools/variant_ab.sh
