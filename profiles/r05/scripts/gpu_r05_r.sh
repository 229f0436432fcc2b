#!/bin/bash
# fp64 small kernels in their own unit with MachineLICM on: the whole GPU
# suite, then config #2 (and #5 as a control) against the build without it.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05r}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread > "$O/pytest_all.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/pytest_all.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TAG=${TAG:-r05r}/ab VARIANTS="f64s_nolicm" CFGS="2 5" REPS=3 bash tools/variant_ab.sh | tee "$O/ab.txt"
