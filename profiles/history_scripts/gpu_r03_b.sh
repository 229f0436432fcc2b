set -u
bash tools/mcse_dump.sh || exit 1
timeout -k 10 300 tools/fdiv_exhaust 64 > gpurun_out/fdiv_exhaust.txt 2>&1; echo fdiv rc=$?; cat gpurun_out/fdiv_exhaust.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routines.py tests/test_bench_launch.py tests/test_gpu_driver.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r03b.log 2>&1; echo pytest rc=$?; tail -4 gpurun_out/pytest_gpu_r03b.log
TAG=ldsw VARIANTS="ldswait0 fdiv7" CFGS=3 REPS=2 bash tools/variant_ab.sh
