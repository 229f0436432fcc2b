#!/bin/bash
# Per-phase wave-cycle split (tools/phase_profile.py, lib_phase variant) and the
# SQ issue/wait split of the default bench (tools/pmc_sq.sh).  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-phase}; mkdir -p "$OUT"
timeout -k 10 300 python tools/phase_profile.py 1048576 mixed ref lon-snow-type > "$OUT/phase_mixed.txt" 2>&1 || { tail -5 "$OUT/phase_mixed.txt"; exit 1; }
cat "$OUT/phase_mixed.txt"
timeout -k 10 300 python tools/phase_profile.py 1048576 mixed ref as-generated > "$OUT/phase_mixed_gen.txt" 2>&1 || { tail -5 "$OUT/phase_mixed_gen.txt"; exit 1; }
cat "$OUT/phase_mixed_gen.txt"
TAG=${TAG:-phase}_sq bash tools/pmc_sq.sh
