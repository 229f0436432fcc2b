#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the default bench for one library
# (LIB=variant name or "default"), --kernel-trace only.  GPU box.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
LIBN=${LIB:-default}
OUT="$R/gpurun_out/${TAG:-pmcv}/$LIBN"
mkdir -p "$OUT"
if [ "$LIBN" = default ]; then export NOAHMP_ENGINE_LIB=""; else export NOAHMP_ENGINE_LIB="$R/noahmp-1_amd/lib/variants/lib_$LIBN.so"; fi
cd /tmp && export TMPDIR=/tmp
[ -x "$R/tools/calib_copy" ] || hipcc -O3 --offload-arch=gfx950 -o "$R/tools/calib_copy" "$R/tools/calib_copy.hip" || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  [ -d "$R/gpurun_out/${TAG:-pmcv}/calib_$C" ] || { timeout -k 10 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG:-pmcv}/calib_$C" -o run -- "$R/tools/calib_copy" 4194304 3 > "$OUT/calib_$C.log" 2>&1 || exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/bench_$C" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_$C.log" 2>&1
  rc=$?; echo "$LIBN $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
