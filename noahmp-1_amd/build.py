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
DEFAULT_LIB_PATH = os.path.join(LIB_DIR, "libnoahmp_engine.so")
# NOAHMP_ENGINE_LIB: a tuning variant (tools/build_variants.py), hash-checked only on request
LIB_PATH = os.environ.get("NOAHMP_ENGINE_LIB") or DEFAULT_LIB_PATH
SOURCES = ["engine.hip", "sflx_kernel.hip", "sflx_kernel_f64.hip", "sflx_kernel_f64s.hip",
           "rebin.hip", "forcing.hip", "routines.hip", "tables.cpp"]
HEADERS = ["dev_params.h", "sflx_kargs.h", "sflx_math.h", "sflx_routines.h", "glibc_math.h",
           "vege_domain.h"]
# per-source flags: sflx_kernel.hip is compiled as the fp32 translation unit,
# sflx_kernel_f64.hip (the same file, NMP_TU 8) as the fp64 one, in parallel.
# The fp64 unit can take its own flags (tools/build_variants.py f64*): with
# -freciprocal-math or -fapprox-func its divisions outside the Newton loops
# become reciprocal sequences, which measured no faster on configs #2/#5
# (profiles/r02/f64_flags_ab.txt), so it builds with the common flags.
# fp32 translation unit: no SimplifyCFG sinking of instructions common to both
# arms of a branch (config #3 +0.95 % over 4 interleaved A/B rounds; the fp64
# kernels measured -1 % with it, profiles/r02/f32only_ab.txt)
# MachineLICM hoists uniform offsets/constants out of the step and Newton
# loops and holds them across the whole step: spills 70 -> 42 (single-step
# kernel) without it; with the round-5 addressing it still costs config #3
# 2.6 % and config #5 9 %, but gives config #2's fp64 one-wave-per-SIMD
# kernel +2 % (profiles/r05/retune_ab.txt): on for that translation unit only
_LICM_OFF = ["-mllvm", "-disable-machine-licm"]
SOURCE_FLAGS = {src: list(_LICM_OFF) for src in SOURCES}
SOURCE_FLAGS["sflx_kernel.hip"] = ["-DNMP_TU=4", "-mllvm", "-simplifycfg-sink-common=false",
                                   *_LICM_OFF]
SOURCE_FLAGS["sflx_kernel_f64s.hip"] = []
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-std=c++17",
         "-ffp-contract=off", "-Wno-unused-result", "-Wno-unused-value",
         # (MachineLICM: off per source, SOURCE_FLAGS)
         # no SLP vectorizer: the packed f32 ops it forms (v_pk_fma/mul/add,
         # same IEEE result per element) need aligned register pairs; without
         # them the fp32 step kernel spills 37 VGPRs instead of 52 (scratch
         # 168 -> 124 B/lane) and config #3 runs +2.3 % (profiles/r02/noslp_ab.txt)
         "-fno-slp-vectorize",
         # no scalar partial-redundancy elimination (GVN-PRE): fewer values
         # kept live across branches; config #3 +0.7 %, config #5 +1.3 %
         # (profiles/r02/flags3_ab.txt)
         "-mllvm", "-enable-pre=false"]


def source_hash(extra: tuple = (), source_flags: dict | None = None) -> str:
    """Hash of every engine source + build flag: identifies the kernel a
    measurement (profiles/traffic.json) was taken on.  Compiled into the
    library (nmp_build_hash), so a stale library is detected at load time."""
    import hashlib
    h = hashlib.sha256(" ".join(FLAGS + list(extra)).encode())
    h.update(repr(sorted((source_flags or SOURCE_FLAGS).items())).encode())
    for p in sorted(SOURCES + HEADERS):
        with open(os.path.join(CSRC, p), "rb") as f:
            h.update(f.read())
    with open(os.path.join(ROOT, "include", "noahmp_engine.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def built_hash(path: str = LIB_PATH) -> str | None:
    """The source hash compiled into the library at `path` (read from the file,
    without loading it), or None if there is no library or no marker."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    i = data.find(b"NMP_BUILD_HASH=")
    return data[i + 15:i + 31].decode() if i >= 0 else None


LLVM_MC = os.environ.get("LLVM_MC", "/opt/rocm/lib/llvm/bin/llvm-mc")


def check_device_asm(asm_files, verbose: bool = True):
    """Re-assemble the compiler's own device assembly text with llvm-mc and fail
    on any instruction it rejects.  The integrated assembler does not reject
    them: it encodes what it can.  ROCm 7.2's LLVM, for one, can select an
    `s_mov_b64` of a 64-bit immediate that gfx950 cannot encode, and the object
    then silently holds the literal's low 32 bits (tools/llvm_repro/: the fp64
    kernels built without MachineCSE computed exp(x) = inf for x > 0, VERDICT
    r2 item 1).  A build whose text does not assemble is refused."""
    if not os.path.exists(LLVM_MC):
        raise RuntimeError(f"device assembly check: llvm-mc not found at {LLVM_MC} (set LLVM_MC "
                           "to its path, or build with check_asm=False)")
    bad = []
    for a in asm_files:
        r = subprocess.run([LLVM_MC, "-triple=amdgcn-amd-amdhsa", f"-mcpu={ARCH}", "-filetype=null",
                            a], capture_output=True, text=True)
        if r.returncode != 0:
            errs = [ln for ln in r.stderr.splitlines() if "error:" in ln]
            bad.append(f"{os.path.basename(a)}: {len(errs)} unencodable instructions, e.g. "
                       f"{errs[0] if errs else r.stderr[:200]}")
    if bad:
        raise RuntimeError("device assembly check failed (the object would not hold what the "
                           "compiler selected):\n" + "\n".join(bad))
    check_kernarg_layout(asm_files)
    if verbose:
        print(f"[noahmp build] device asm re-assembles cleanly ({len(asm_files)} units)", flush=True)


def check_kernarg_layout(asm_files):
    """The fp32 step kernels re-read their array bases from the kernel-argument
    segment at KArgs' byte offset 8 (sflx_kernel.hip kargs_seg, NMP_OFF32=3).
    Every sflx_step_kernel's code-object metadata must place its second
    argument (KArgs, by value) at offset 8; a build where it does not is
    refused."""
    import re
    bad = []
    for a in asm_files:
        text = open(a).read()
        for m in re.finditer(r"\.args:(.*?)\.name:\s+(\S+)", text, re.S):
            if "sflx_step_kernel" not in m.group(2):
                continue
            offs = re.findall(r"\.offset:\s+(\d+)", m.group(1))
            if len(offs) < 2 or offs[1] != "8":
                bad.append(f"{m.group(2)}: argument offsets {offs[:2]}")
    if bad:
        raise RuntimeError("kernel-argument layout check failed (KArgs not at byte offset 8):\n"
                           + "\n".join(bad))


def build(force: bool = False, verbose: bool = True, out: str | None = None,
          extra: tuple = (), source_flags: dict | None = None, check_asm: bool = True) -> str:
    """Build the engine library (default: LIB_PATH; `out`/`extra`/`source_flags`
    for tuning variants).  check_asm: also emit each HIP unit's device assembly
    and re-assemble it (check_device_asm)."""
    path = out or LIB_PATH
    sflags = source_flags or SOURCE_FLAGS
    want = source_hash(extra, sflags)
    if not force and built_hash(path) == want:
        return path
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = path + ".tmp"
    objdir = tmp + ".objs"
    os.makedirs(objdir, exist_ok=True)
    inc = ["-I", os.path.join(ROOT, "include"), "-I", CSRC]
    cmds = []
    for src in SOURCES:
        obj = os.path.join(objdir, src + ".o")
        cflags = [f for f in FLAGS if f != "-shared"]
        cmds.append((obj, [HIPCC, *cflags, *sflags.get(src, []), *extra,
                           f'-DNMP_BUILD_HASH="{want}"', *inc, "-c", "-o", obj,
                           os.path.join(CSRC, src)]))
    asm = []
    if check_asm:
        for src in SOURCES:
            if not src.endswith(".hip"):
                continue
            a = os.path.join(objdir, src + ".s")
            cflags = [f for f in FLAGS if f not in ("-shared", "-fPIC")]
            asm.append((a, [HIPCC, *cflags, *sflags.get(src, []), *extra,
                            f'-DNMP_BUILD_HASH="{want}"', *inc, "--offload-device-only", "-S",
                            "-o", a, os.path.join(CSRC, src)]))
    if verbose:
        for _, c in cmds:
            print("[noahmp build]", " ".join(c), flush=True)
    from concurrent.futures import ThreadPoolExecutor
    asm_cmds = [x for _, x in asm]

    def compile_one(c):
        # the asm pass is quiet unless it fails; then its diagnostics are shown
        quiet = c in asm_cmds
        r = subprocess.run(c, capture_output=quiet, text=True)
        if r.returncode != 0:
            if quiet:
                sys.stderr.write(r.stdout + r.stderr)
            raise subprocess.CalledProcessError(r.returncode, c)

    jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(cmds) + len(asm), os.cpu_count() or 1)
    with ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(compile_one, c) for _, c in cmds + asm]:
            f.result()
    if asm:
        check_device_asm([a for a, _ in asm], verbose)
    link = [HIPCC, *FLAGS, *extra, "-o", tmp, *[o for o, _ in cmds]]
    if verbose:
        print("[noahmp build]", " ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(tmp, path)
    import shutil
    shutil.rmtree(objdir, ignore_errors=True)
    return path


if __name__ == "__main__":
    build(force="--force" in sys.argv)
