#!/bin/bash
# Rehearsal of bench.py's N>1 control flow on a one-GPU box: torchrun with 2
# and 4 ranks sharing the device over gloo (NMP_BENCH_BACKEND=gloo; RCCL
# refuses two ranks on one device), gather to root and all-gather, output every
# 6th step and every step.  Checks that rank 0 prints one JSON line with
# n_gpus = N and clean status; the numbers are not measurements.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-dist}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NMP_BENCH_BACKEND=gloo
port=29561
for spec in "2 root 6" "2 all 1" "4 root 1" "4 all 6"; do
  set -- $spec
  log="$OUT/n$1_$2_out$3.log"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $1 --no-cpu-baseline \
    --ncol 65536 --steps 12 --warmup 2 --gather $2 --out-every $3 > "$log" 2>&1
  rc=$?; port=$((port + 1))
  echo "== N=$1 gather=$2 out_every=$3 rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$log"; exit $rc; }
  python - "$log" $1 <<'EOF'
import json, sys
lines = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')]
assert len(lines) == 1, f"{len(lines)} JSON lines"
d = json.loads(lines[0])
assert d["n_gpus"] == int(sys.argv[2]) and d["checks"]["status_nonzero_cols"] == 0 and d["checks"]["stc_finite"], d
print("ok", d["n_gpus"], d["config"]["ncol_total"], d["config"]["gather"], d["config"]["backend"], round(d["value"] / 1e6, 1))
EOF
  [ $? -eq 0 ] || exit 1
done
