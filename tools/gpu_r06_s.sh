#!/bin/bash
# Round 6, box S: the file-format kernels' launch times and HBM bandwidth
# (tools/io_kernels_bench.py, HIP events, then rocprofv3 kernel statistics of
# the same run), and the argument-check GPU test of their entries.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=$R/gpurun_out/${TAG:-r06s}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_forcing.py -m gpu -q --timeout 240 \
  --timeout-method thread > "$O/pytest_forcing.log" 2>&1 || { tail -5 "$O/pytest_forcing.log"; exit 1; }
tail -1 "$O/pytest_forcing.log"
timeout -k 10 300 python -u tools/io_kernels_bench.py > "$O/io_kernels.json" 2>&1 || exit $?
cat "$O/io_kernels.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/tools/io_kernels_bench.py" > "$O/prof.log" 2>&1 || exit $?
echo done
