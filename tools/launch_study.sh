#!/bin/bash
# Config #4's launch-size effect: the 4,194,304-column
# CONUS set as one launch per stream range, the same set as sequential
# 262,144-column launches (the per-launch size of a 524,288-column shard on 2
# ranges), the 524,288-column shard itself, and that shard tiled 8x into one
# 4 M launch set.  Interleaved twice; one JSON line per run under $O.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05_launch}
mkdir -p "$O"
B="python -u bench.py --kind conus --steps ${STEPS:-20} --warmup 5 --period 8 --no-cpu-baseline"
for rep in 1 2; do
  for cfg in "full:--ncol 4194304" "seq262k:--ncol 4194304 --launch-cols 262144" \
             "shard:--ncol 524288" "tiled8:--ncol 4194304 --replicate 8" \
             "shard_s4:--ncol 524288 --streams 4" "full_seq524k:--ncol 4194304 --launch-cols 524288"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 240 $B $args > "$O/${name}_$rep.log" 2>&1
    rc=$?; v=$(grep '^{' "$O/${name}_$rep.log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4))" 2>/dev/null)
    echo "$name rep$rep rc=$rc Mcs/s ms/step: $v" | tee -a "$O/summary.txt"
    [ $rc -eq 0 ] || exit $rc
  done
done
