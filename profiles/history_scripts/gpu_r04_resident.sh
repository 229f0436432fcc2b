#!/bin/bash
# Round 4: resident launches (work-queue chunks).  GPU box: the GPU suite on
# the new default build, then an interleaved config #3 A/B against the same
# library with resident launches off and the previous commit's build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04_res}; mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
fi
TAG=${TAG:-r04_res} VARIANTS="${VARIANTS:-default@NMP_RESIDENT=0 prev}" CFGS="${CFGS:-3}" REPS="${REPS:-3}" \
  bash tools/variant_ab.sh | tee "$OUT/ab.txt"
