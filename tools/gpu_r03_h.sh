#!/bin/bash
# fast division with the fallback kernel: fixture parity (default, always-
# fallback fd3, guard probes g1/g2), the forced re-run tests, then an A/B on
# config #3 / #5 against fd2 (no guard) and fd0 (IEEE division).  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/fdiag
VARIANTS="default fd3 g1 g2" bash tools/gpu_r03_f.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "fast_division or order_check" -s > gpurun_out/fdiv_tests2.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "re-runs|passed|failed|differ" gpurun_out/fdiv_tests2.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
TAG=fdivab2 VARIANTS="g1 g2 fd2 fd0" CFGS="3" REPS=2 bash tools/variant_ab.sh
