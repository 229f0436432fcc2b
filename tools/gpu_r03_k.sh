#!/bin/bash
# stream-shard scenario, step by step, on the fast-division builds:
# fd1 (guarded) and fd3 (every wave re-runs with the reference divisions)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS:-fd3 fd1}; do
  NOAHMP_ENGINE_LIB=$PWD/noahmp-1_amd/lib/variants/lib_$v.so timeout -k 10 300 python -u tools/fdiv_shard_diag.py 2 > gpurun_out/fdiv_shard_diag_$v.txt 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v "^    \[" gpurun_out/fdiv_shard_diag_$v.txt | grep -v amdgpu.ids | head -12
  [ $rc -le 1 ] || exit $rc
done
