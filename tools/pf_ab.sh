#!/bin/bash
# Layer-state LDS copy: parity tests on the default library, then config #3
# A/B against the variants (nopf = no copy, pf1 = entry reads only, pf2 =
# re-read only).  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-pf}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$OUT/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 "$OUT/parity.log"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-pf}/ab VARIANTS="${VARIANTS:-nopf pf1 pf2}" CFGS=3 REPS=${REPS:-2} bash tools/variant_ab.sh
