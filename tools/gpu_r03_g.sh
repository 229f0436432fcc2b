#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/fdiag
timeout -k 10 120 python -u tools/fdiv_cols.py combo_r2 75 89 > gpurun_out/fdiag/cols_default.txt 2>&1 || exit 1
NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_fd2.so timeout -k 10 120 python -u tools/fdiv_cols.py combo_r2 75 89 > gpurun_out/fdiag/cols_fd2.txt 2>&1 || exit 1
echo ok
