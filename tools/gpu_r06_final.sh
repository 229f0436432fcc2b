#!/bin/bash
# Round 6 closing check on the final tree: the whole GPU suite and smoke.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06fin}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > "$O/pytest_all.log" 2>&1 || { echo "pytest rc=$?"; tail -15 "$O/pytest_all.log"; exit 1; }
tail -2 "$O/pytest_all.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -5 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
echo done
