#!/bin/bash
# Wave-slot occupancy over a step (tools/wave_timeline.py) for the default
# block (256) at 1 and 2 stream ranges and for 128/64-column blocks, then an
# A/B of the 128/64 blocks (no LDS state copy) on config #3.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-wave}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for spec in "wt 1" "wt 2" "wt_b128 2" "wt_b64 2"; do
  set -- $spec
  timeout -k 10 180 python tools/wave_timeline.py $1 $2 6 > "$OUT/tl_$1_s$2.txt" 2>&1
  rc=$?; echo "== $1 streams=$2 rc=$rc"; grep -v amdgpu.ids "$OUT/tl_$1_s$2.txt" | tail -8
  [ $rc -eq 0 ] || exit $rc
done
TAG=${TAG:-wave}/ab VARIANTS="${VARIANTS:-b128_nopf b64_nopf}" CFGS="3" REPS=2 bash tools/variant_ab.sh
