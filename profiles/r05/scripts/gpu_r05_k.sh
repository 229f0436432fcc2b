#!/bin/bash
# 32-bit column offsets: the whole GPU suite on the new default library, then
# an interleaved A/B against the 64-bit-pointer build (off64) on configs 3, 5, 2.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05k}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread > "$O/pytest_all.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/pytest_all.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TAG=r05k/ab VARIANTS="off64" CFGS="3 5 2" REPS=3 bash tools/variant_ab.sh | tee "$O/ab.txt"
