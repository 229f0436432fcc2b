#!/bin/bash
# Round 4: how much of the step is launch tail -- the bench workload per
# column at 1, 2 and 4 M columns, and 1 M columns over 1-4 stream ranges.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04_scale; mkdir -p "$OUT"
run() { local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 48 --warmup 4 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -3 "$OUT/$name.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']/1e6,1), 'Mcs/s step_ms', round(d['roofline']['step_ms'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],4))"; }
for s in 1 2 3 4; do run m1_s$s --streams $s; done
run m2_s2 --ncol 2097152 --period 16
run m4_s2 --ncol 4194304 --period 8
run m4_s1 --ncol 4194304 --period 8 --streams 1
run m1_s2_again
