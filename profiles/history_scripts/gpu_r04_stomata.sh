#!/bin/bash
# Round 4: range-proved short division in the stomata bisection.  GPU box:
# the GPU suite, an interleaved config #3 A/B (previous build, unguarded probe),
# and the IEEE-path rates on the bench column sets (fbcount build).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04_sto}; mkdir -p "$OUT"
TAG=${TAG:-r04_sto} VARIANTS="prev stfast" CFGS="${CFGS:-3}" REPS="${REPS:-3}" bash tools/gpu_r04_resident.sh || exit 1
NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_fbcount.so timeout -k 10 300 python tools/fallback_rate.py > "$OUT/fallback_rate.txt" 2>&1 || { tail -5 "$OUT/fallback_rate.txt"; exit 1; }
cat "$OUT/fallback_rate.txt"
