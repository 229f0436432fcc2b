#!/bin/bash
# checkpoint values (NMP_DEBUG_DUMP) of a few columns from the
# debug build with and without MachineCSE in the fp64 unit (tools/mcse_probe.py dump).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/mcse"
mkdir -p "$OUT"
for V in dbg64 nomcse64_dbg; do
  NOAHMP_ENGINE_LIB="$R/noahmp-1_amd/lib/variants/lib_$V.so" timeout -k 10 240 python3 -u "$R/tools/mcse_probe.py" dump "$OUT/dump_$V.npz" > "$OUT/dump_$V.log" 2>&1 || { echo "$V dump failed"; tail -5 "$OUT/dump_$V.log"; exit 1; }
done
python3 "$R/tools/mcse_probe.py" cmpdump "$OUT/dump_dbg64.npz" "$OUT/dump_nomcse64_dbg.npz" > "$OUT/dump_report.txt" 2>&1
grep -c differs "$OUT/dump_report.txt"
exit 0
