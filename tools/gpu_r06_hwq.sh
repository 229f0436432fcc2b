#!/bin/bash
# Round 6: stream ranges x hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4)
# on config #3 with the driver's window, interleaved, 2 rounds.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06hwq}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
run() {  # name queues streams
  local name=$1 q=$2 s=$3
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --streams $s > "$O/$name.log" 2>&1 || { echo "$name rc=$?"; tail -3 "$O/$name.log"; exit 1; }
  python -c "import json; d=[json.loads(l) for l in open('$O/$name.log') if l.startswith('{\"metric')][-1]; print('$name', round(d['value']/1e6,1), 'Mcs/s', round(d['ms_per_step'],4))" | tee -a "$O/ab.txt"
}
for rep in 1 2; do
  run q4s2_$rep 4 2
  run q8s2_$rep 8 2
  run q8s3_$rep 8 3
  run q8s4_$rep 8 4
  run q8s6_$rep 8 6
  run q4s4_$rep 4 4
done
echo done
