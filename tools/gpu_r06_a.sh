#!/bin/bash
# Round 6, first box: config #3 with the driver's arguments (this box's
# reference), then config #5 as the 8-GPU run holds it -- each of the 8
# shards of 129,600 fp64 columns (carbon on, hourly, output every step,
# forcing generated on the device) stepped alone on this GPU -- and the
# RCCL gather's own cost at world 1 (forced collective) under torchrun.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06a}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
summ() {  # name
  python -c "import json,sys; d=[json.loads(l) for l in open('$O/$1.log') if l.startswith('{\"metric')][-1]; r=d['roofline']; print('$1', round(d['value']/1e6,1), 'Mcs/s ms/step', round(d['ms_per_step'],4), 'gpu_step_ms', round(r['step_ms'],4), 'kern_ms', round(r['kernel_ms'],4))" | tee -a "$O/summary.txt"
}
run() {  # name args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 "$O/$name.log"; exit $rc; }
  summ "$name"
}
CFG5="--kind global --ncol 129600 --precision 8 --opt-veg 2 --dt 3600 --out-every 1 --forcing device"
run cfg3_driver_1 --steps 20 --warmup 5
for r in 0 1 2 3 4 5 6 7; do
  run cfg5_shard_r$r $CFG5 --emulate-rank $r --steps 48 --warmup 4
done
run cfg5_shard_r3_s1 $CFG5 --emulate-rank 3 --steps 48 --warmup 4 --streams 1
run cfg5_shard_r3_noout $CFG5 --emulate-rank 3 --steps 48 --warmup 4 --out-every 1000
port=29571
for g in all root; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --no-cpu-baseline \
    $CFG5 --steps 48 --warmup 4 --gather $g --force-collective > "$O/cfg5_n1_force_$g.log" 2>&1
  rc=$?; port=$((port + 1))
  [ $rc -eq 0 ] || { echo "force $g rc=$rc"; tail -5 "$O/cfg5_n1_force_$g.log"; exit $rc; }
  summ cfg5_n1_force_$g
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --no-cpu-baseline \
  $CFG5 --steps 48 --warmup 4 > "$O/cfg5_n1_plain.log" 2>&1 || { echo "n1 plain failed"; exit 1; }
summ cfg5_n1_plain
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_cfg5" -o run -- \
  python -u "$R/bench.py" --no-cpu-baseline $CFG5 --emulate-rank 3 --steps 20 --warmup 4 \
  > "$O/prof_cfg5.log" 2>&1 || { echo "rocprof cfg5 failed"; tail -5 "$O/prof_cfg5.log"; exit 1; }
cd "$R"
run cfg3_driver_2 --steps 20 --warmup 5
echo done
