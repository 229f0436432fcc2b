#!/bin/bash
# Round-2 evidence pass (GPU box): gpu tests, smoke, PMC traffic passes and a
# kernel-trace summary of the default bench, the default bench line (with the
# CPU baseline), and a torchrun N=1 bench over RCCL.  Every GPU step is
# time-limited; a failure ends the script.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
TAG=${TAG:-r02final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -1 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG}_pmc VALU=1 bash tools/pmc_run.sh > "$OUT/pmc.log" 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc.log"; exit $rc; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/ktrace" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$R/$OUT/ktrace.log" 2>&1)
rc=$?; echo "ktrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --no-cpu-baseline > "$OUT/bench_dist_n1.log" 2>&1
rc=$?; echo "torchrun bench rc=$rc"; tail -1 "$OUT/bench_dist_n1.log"; [ $rc -eq 0 ] || exit $rc
