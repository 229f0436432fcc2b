#!/bin/bash
# Round 4: where the range-checked canopy division loses its gain -- fallback
# causes, and A/B of probe builds that drop one part of the check each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04_div2; mkdir -p "$OUT"
NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_fbcount.so timeout -k 10 300 \
  python tools/fallback_rate.py > "$OUT/fallback_rate.txt" 2>&1 || { echo "fallback probe failed"; tail "$OUT/fallback_rate.txt"; exit 1; }
cat "$OUT/fallback_rate.txt"
TAG=r04_div2/ab VARIANTS="vd0 vdnodom vdnowin vdallfast vdnone" CFGS="3" REPS=2 bash tools/variant_ab.sh > "$OUT/ab.txt" 2>&1
cat "$OUT/ab.txt"
