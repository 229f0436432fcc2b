#!/bin/bash
# Interleaved sunlit/shaded stomata solves (stpair variant): parity tests on
# the variant library, then an A/B against the default on config #3.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r05bb}
mkdir -p "$O"
NOAHMP_ENGINE_LIB=$R/noahmp-1_amd/lib/variants/lib_stpair.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 120 --timeout-method thread > "$O/pytest_stpair.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/pytest_stpair.log"
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05bb}/ab VARIANTS="stpair" CFGS="3" REPS=4 bash tools/variant_ab.sh | tee "$O/ab.txt"
