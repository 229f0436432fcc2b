#!/bin/bash
# Round 4: the whole-step IEEE re-run (kPassRerun) in place of the in-loop
# re-run.  GPU box: the full GPU suite on the new default build, then an
# interleaved A/B on config #3 against the previous build (lib_prev, the
# in-loop re-run) and the no-fallback probe (lib_vdnofb).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04_rerun; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
TAG=r04_rerun VARIANTS="${VARIANTS:-prev vdnofb}" CFGS="3" REPS="${REPS:-3}" bash tools/variant_ab.sh \
  | tee "$OUT/ab.txt"
