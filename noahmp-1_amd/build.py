"""In-tree build of libnoahmp_engine.so for gfx950 (hipcc).

The library holds the HIP column kernel (csrc/sflx_kernel.hip), the C ABI
(csrc/engine.hip) and the TBL reader (csrc/tables.cpp).  It is built into
noahmp-1_amd/lib/ so it travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libnoahmp_engine.so")
SOURCES = ["engine.hip", "sflx_kernel.hip", "tables.cpp"]
HEADERS = ["dev_params.h", "sflx_kargs.h", "sflx_math.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-std=c++17",
         "-ffp-contract=off", "-Wno-unused-result", "-Wno-unused-value"]


def _newest_input() -> float:
    paths = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    paths.append(os.path.join(ROOT, "include", "noahmp_engine.h"))
    paths.append(os.path.abspath(__file__))
    return max(os.path.getmtime(p) for p in paths)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= _newest_input():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC, *FLAGS, "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-o", tmp,
           *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        print("[noahmp build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    build(force="--force" in sys.argv)
