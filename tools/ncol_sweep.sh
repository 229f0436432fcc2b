#!/bin/bash
# Config #3's kind at column counts from 65,536 to 16,777,216 on one GPU: the
# throughput curve of the engine against problem size (launch ramp and drain
# amortised, the 288-GB HBM used), the driver's 20-after-5 window.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-ncol_sweep}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
for n in 65536 131072 262144 524288 1048576 2097152 4194304 8388608 16777216; do
  p=48; [ $n -gt 4194304 ] && p=8
  timeout -k 10 300 python -u bench.py --ncol $n --period $p --steps 20 --warmup 5 --no-cpu-baseline > "$O/n$n.log" 2>&1 || { echo "n=$n rc=$?"; tail -3 "$O/n$n.log"; exit 1; }
  python -c "import json; d=[json.loads(l) for l in open('$O/n$n.log') if l.startswith('{\"metric')][-1]; r=d['roofline']; print($n, round(d['value']/1e6,1), 'Mcs/s', round(d['ms_per_step'],4), 'ms/step', 'frac', round(r['frac'],4))" | tee -a "$O/sweep.txt"
done
echo done
