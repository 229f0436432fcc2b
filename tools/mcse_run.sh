#!/bin/bash
# VERDICT r2 item 1 on the GPU box: fp64 results of a library variant against
# the shipped library (tools/mcse_probe.py).  VARIANT=nomcse64 by default.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
V="${VARIANT:-nomcse64}"
OUT="$R/gpurun_out/mcse"
mkdir -p "$OUT"
T=$(mktemp -d)
timeout -k 10 240 python3 -u "$R/tools/mcse_probe.py" run "$T/base.npz" ${PROBE_ARGS:-} > "$OUT/run_base.log" 2>&1 || { echo "base run failed"; tail -5 "$OUT/run_base.log"; exit 1; }
NOAHMP_ENGINE_LIB="$R/noahmp-1_amd/lib/variants/lib_$V.so" timeout -k 10 240 python3 -u "$R/tools/mcse_probe.py" run "$T/$V.npz" ${PROBE_ARGS:-} > "$OUT/run_$V.log" 2>&1 || { echo "$V run failed"; tail -5 "$OUT/run_$V.log"; exit 1; }
python3 "$R/tools/mcse_probe.py" cmp "$T/base.npz" "$T/$V.npz" > "$OUT/report_$V.txt" 2>&1
rc=$?
rm -rf "$T"
cat "$OUT/report_$V.txt" | head -120
exit $rc
