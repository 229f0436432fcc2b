#!/bin/bash
# Round 6, box R: the full-size year sample against the reference (config
# #5's grid, fp32, 8,784 hourly steps), then the bench line five times on one
# box (run-to-run spread of the driver's window, for reading A/B results).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06r}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 560 \
  --timeout-method thread -k full_size_year > "$O/pytest_year.log" 2>&1 || { echo "year test rc=$?"; tail -5 "$O/pytest_year.log"; exit 1; }
tail -3 "$O/pytest_year.log"
for i in 1 2 3 4 5; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_$i.log" 2>&1 || exit $?
  python -c "import json; d=[json.loads(l) for l in open('$O/bench_$i.log') if l.startswith('{\"metric')][-1]; print('run $i', round(d['value']/1e6,1), 'Mcs/s', round(d['ms_per_step'],4), 'ms/step')" | tee -a "$O/repeat.txt"
done
echo done
