"""csrc/glibc_math.h (the kernel's "ref" math) vs the host glibc float libm.

The header is __host__ __device__; here it is compiled for the host with the
same -ffp-contract=off and compared bit for bit against libm.  Default run:
every 61st of the 2^32 float patterns per univariate function, powf on a
stride x 30 exponents + random pairs.  NMP_EXHAUSTIVE=1 checks all 2^32
(each function ~6 s on 8 cores; the committed design claims were made with
that run: 0 mismatches for every function, powf 0 of 2.6e10).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "glibc_math_check.cpp")
FUNCS = ["expf", "exp2f", "logf", "expm1f", "tanhf", "atanf", "log10f", "acosf", "cosf", "tanf"]


@pytest.fixture(scope="module", params=[0, 1], ids=["branches", "branchless"])
def checker(request, tmp_path_factory):
    """The header as compiled by default and with NMP_GM_BRANCHLESS=1 (the
    special-case exits of expf/logf as selects)."""
    exe = str(tmp_path_factory.mktemp("gm") / "glibc_math_check")
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-std=c++17",
                    f"-DNMP_GM_BRANCHLESS={request.param}",
                    "-I", os.path.join(ROOT, "noahmp-1_amd", "csrc"), "-o", exe, SRC, "-lm"],
                   check=True)
    return exe


def _stride(default):
    return "1" if os.environ.get("NMP_EXHAUSTIVE") == "1" else str(default)


@pytest.mark.parametrize("fn", FUNCS)
def test_bit_exact_vs_host_libm(checker, fn):
    r = subprocess.run([checker, fn, _stride(61)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and " mismatches 0 of " in r.stdout, r.stdout + r.stderr


def test_powf_bit_exact_vs_host_libm(checker):
    r = subprocess.run([checker, "powf", _stride(997)], capture_output=True, text=True,
                       timeout=1200)
    assert r.returncode == 0 and " mismatches 0 of " in r.stdout, r.stdout + r.stderr


def test_powf_pair_bit_exact_vs_host_libm(checker):
    """gm::powf_pair (one log2 of the base for two exponents) == two host powf."""
    r = subprocess.run([checker, "powf_pair", _stride(997)], capture_output=True, text=True,
                       timeout=1200)
    assert r.returncode == 0 and " mismatches 0 of " in r.stdout, r.stdout + r.stderr
