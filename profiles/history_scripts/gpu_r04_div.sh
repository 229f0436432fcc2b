#!/bin/bash
# Round 4: the range-proved short division in the canopy loop -- the GPU
# suite on the new default, the fallback rate, and an interleaved A/B against
# the IEEE-only build (vd0).  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04_div; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_fbcount.so timeout -k 10 300 \
  python tools/fallback_rate.py > "$OUT/fallback_rate.txt" 2>&1 || { echo "fallback probe failed"; tail "$OUT/fallback_rate.txt"; exit 1; }
cat "$OUT/fallback_rate.txt"
TAG=r04_div/ab VARIANTS="vd0 bare0" CFGS="3 5" REPS=2 bash tools/variant_ab.sh > "$OUT/ab.txt" 2>&1
cat "$OUT/ab.txt"
