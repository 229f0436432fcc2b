#!/bin/bash
# fast-division diagnosis on the single-call fixtures (GPU box):
# VARIANTS="default fd2 fd0 generic fd3 fd3nf"
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/fdiag
V=noahmp-1_amd/lib/variants
for v in ${VARIANTS:-default fd2 fd0 generic}; do
  case $v in
    default) timeout -k 10 200 python -u tools/fdiv_diag.py > gpurun_out/fdiag/$v.txt 2>&1 ;;
    generic) NMP_GENERIC_OPTIONS=1 timeout -k 10 200 python -u tools/fdiv_diag.py > gpurun_out/fdiag/$v.txt 2>&1 ;;
    *) NOAHMP_ENGINE_LIB=$PWD/$V/lib_$v.so timeout -k 10 200 python -u tools/fdiv_diag.py > gpurun_out/fdiag/$v.txt 2>&1 ;;
  esac
  rc=$?; echo "== $v rc=$rc"; grep -v " bad=0 " gpurun_out/fdiag/$v.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
done
