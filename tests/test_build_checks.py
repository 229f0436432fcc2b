"""Build-time guard against silently mis-encoded device code.

ROCm 7.2's LLVM can select, for gfx950, an `s_mov_b64` of a 64-bit immediate
that the ISA cannot encode; the integrated assembler then keeps only the low 32
bits (tools/llvm_repro/).  build.check_device_asm re-assembles the compiler's
own text output with llvm-mc, which rejects such instructions, and build()
refuses a library whose device code fails it."""
import os
import subprocess

import pytest

import noahmp_pkg  # noqa: F401
from noahmp_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPRO = os.path.join(ROOT, "tools", "llvm_repro", "s_mov_b64_literal.hip")


def _asm(tmp_path, name, flags):
    out = str(tmp_path / f"{name}.s")
    subprocess.run([build.HIPCC, "-O3", f"--offload-arch={build.ARCH}", "--offload-device-only",
                    "-S", "-o", out, REPRO, *flags], check=True, capture_output=True)
    return out


def test_asm_check_rejects_unencodable_literal(tmp_path):
    good = _asm(tmp_path, "default", [])
    build.check_device_asm([good], verbose=False)
    bad = _asm(tmp_path, "nomcse", ["-mllvm", "-disable-machine-cse"])
    with open(bad) as f:
        assert "s_mov_b64 s[0:1], 0x4049000000000000" in f.read()
    with pytest.raises(RuntimeError, match="unencodable"):
        build.check_device_asm([bad], verbose=False)


def test_shipped_library_built_with_asm_check():
    """build() runs the check by default (its signature), and the library in the
    tree is the one built from these sources."""
    import inspect
    assert inspect.signature(build.build).parameters["check_asm"].default is True
    assert build.built_hash() == build.source_hash()
