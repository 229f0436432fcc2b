#!/bin/bash
# Round 6: the bench line on the final build with profiles/traffic.json of
# the same source hash (roofline.traffic / .valu filled): the driver's
# arguments (20 steps after 5) and the default 48 steps.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06q}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_20.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$O/bench_48.log" 2>&1 || exit $?
echo done
