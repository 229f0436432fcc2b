#!/bin/bash
# Rehearsal of the driver's round-end GPU tier on the final tree: the GPU
# suite, smoke, and the default bench line (with its CPU baseline).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06end}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -15 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python -u bench.py > "$O/bench.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$O/bench.log"; exit 1; }
grep '^{"metric' "$O/bench.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e6,1), 'Mcs/s', 'frac', round(r['frac'],4), 'traffic', r.get('traffic') is not None, 'cpu', (d['cpu_baseline'] or {}).get('value'))"
echo done
