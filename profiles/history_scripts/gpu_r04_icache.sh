#!/bin/bash
# Round 4: instruction-cache counters and an interleaved config #3 A/B of
# the default build against variant libraries (LIBS, tools/build_variants.py
# or lib_prev = the previous commit's build).  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_ic}
OUT=gpurun_out/$T; mkdir -p "$OUT"
TAG=$T VARIANTS="${LIBS:-prev norerun}" CFGS="3" REPS="${REPS:-2}" bash tools/variant_ab.sh | tee "$OUT/ab.txt" || exit 1
for v in default ${LIBS:-prev norerun}; do
  if [ "$v" = default ]; then L=""; else L="$PWD/noahmp-1_amd/lib/variants/lib_$v.so"; fi
  NOAHMP_ENGINE_LIB="$L" TAG=$T/ic_$v CTRS="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_IFETCH SQ_BUSY_CYCLES" \
    bash tools/pmc_sq.sh > "$OUT/ic_$v.txt" 2>&1 || { cat "$OUT/ic_$v.txt"; exit 1; }
  echo "== $v"; cat "$OUT/ic_$v.txt"
done
