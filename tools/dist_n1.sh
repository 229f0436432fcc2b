#!/bin/bash
# torchrun N=1 vs plain bench: where the distributed path's overhead comes from.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-distn1}; mkdir -p "$OUT"
run() {  # name, launcher args..., -- bench args
  local name=$1; shift
  timeout -k 10 200 "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e6,1), 'step_ms', round(d['roofline']['step_ms'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],4))"
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
run plain python bench.py --no-cpu-baseline
run plain_noout python bench.py --no-cpu-baseline --out-every 100000
run dist $TR bench.py --gpus 1 --no-cpu-baseline
run dist_noout $TR bench.py --gpus 1 --no-cpu-baseline --out-every 100000
run dist_all $TR bench.py --gpus 1 --no-cpu-baseline --gather all
run plain2 python bench.py --no-cpu-baseline
