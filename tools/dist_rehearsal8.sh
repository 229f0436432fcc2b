#!/bin/bash
# Rehearsal of the driver's N = 8 bench launch on a one-GPU box (VERDICT r5
# item 4): torch.distributed.run with 8 ranks sharing the device over gloo
# (NMP_BENCH_BACKEND=gloo; RCCL refuses two ranks on one device), exactly the
# launch line the driver uses, on config #4's 524,288-column CONUS shards and
# on config #3's column kind at a reduced 131,072 columns per rank, gather to
# root and all-gather.  Checks one JSON line from rank 0 with n_gpus 8, the
# summed column count and finite temperatures.  The rates are not measurements: the
# eight ranks share one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-dist8}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NMP_BENCH_BACKEND=gloo
port=29661
for spec in "conus 524288 all 6" "conus 524288 root 1" "mixed 131072 all 1" "mixed 131072 root 6"; do
  set -- $spec
  log="$OUT/n8_$1_$2_$3_out$4.log"
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --no-cpu-baseline \
    --kind $1 --ncol $2 --period 4 --steps 8 --warmup 2 --gather $3 --out-every $4 > "$log" 2>&1
  rc=$?; port=$((port + 1))
  echo "== N=8 kind=$1 ncol/rank=$2 gather=$3 out_every=$4 rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$log"; exit $rc; }
  python - "$log" 8 $2 <<'EOF'
import json, sys
lines = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')]
assert len(lines) == 1, f"{len(lines)} JSON lines"
d = json.loads(lines[0])
n, per = int(sys.argv[2]), int(sys.argv[3])
assert d["n_gpus"] == n and d["config"]["ncol_total"] == n * per, d
assert d["checks"]["stc_finite"], d
print("ok", d["n_gpus"], d["config"]["ncol_total"], d["config"]["gather"], d["config"]["backend"],
      "status bits on", d["checks"]["status_nonzero_cols"], "cols;",
      round(d["value"] / 1e6, 1), "Mcs/s (8 ranks on one GPU: not a measurement)")
EOF
  [ $? -eq 0 ] || exit 1
done
