#!/bin/bash
# Round 6, final build: the per-phase counters of config #3 again
# (tools/phase_counters.sh on lib_trunc.so, rebuilt from the final sources).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06yy}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
MARKS="3 4 5 6 14 9 10 11 13 99" TAG=${TAG:-r06yy}/phase bash tools/phase_counters.sh || exit 1
cd "$R" && python tools/phase_counters.py "$O/phase" --out "$O/phase_counters.json" --label "config #3 (final build)" > "$O/phase_counters.txt" && cat "$O/phase_counters.txt"
echo done
