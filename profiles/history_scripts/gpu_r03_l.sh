#!/bin/bash
# dget as unconditional pins + selects (default) vs the branchy form (dgetbr):
# all GPU tests on the default build, then an A/B on configs #3 and #5.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_dget.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/gpu_tests_dget.log
[ $rc -eq 0 ] || exit $rc
TAG=dgetab VARIANTS="${VARIANTS:-dgetbr}" CFGS="3 5" REPS=2 bash tools/variant_ab.sh
