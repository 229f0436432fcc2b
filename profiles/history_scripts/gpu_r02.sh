#!/bin/bash
# Round-2 GPU session: gpu tests, smoke, bench (with CPU baseline), torchrun N=1
# bench over RCCL (DiagGather path).  Every GPU step is time-limited; a
# crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r02}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 ${T_TEST:-600} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log"; [ $rc -eq 0 ] || exit $rc
if [ "${DIST:-1}" = 1 ]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --no-cpu-baseline > "$OUT/bench_dist_n1.log" 2>&1
  rc=$?; echo "torchrun bench rc=$rc"; tail -1 "$OUT/bench_dist_n1.log"; [ $rc -eq 0 ] || exit $rc
fi
