"""Shared test setup.

`-m "not gpu"`: oracle vs reference goldens, table reader, ABI/exports, host
logic, gloo sharding.  `-m gpu`: HIP engine parity through the C ABI.
The oracle (oracle/) is test infrastructure: only tests, smoke() and bench's
cpu_baseline leg import it.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import noahmp_pkg  # noqa: E402,F401  (registers noahmp-1_amd as noahmp_amd)

GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle_port():
    """The C restatement (oracle/build/liboracle_f{32,64}.so), built on demand with gcc."""
    import port
    if not all(port.available(p) for p in port.LIBS):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "port"], check=True)
    return port


@pytest.fixture(scope="session")
def engine_lib():
    """The engine C-ABI library (built on demand with hipcc, no fallback).  A
    tuning variant named by NOAHMP_ENGINE_LIB (tools/build_variants.py) is
    loaded as built: rebuilding it here would replace it with the default
    build's flags."""
    from noahmp_amd import build, lib
    if build.LIB_PATH == build.DEFAULT_LIB_PATH:
        build.build()
    return lib.load()


@pytest.fixture(scope="session")
def ref_params():
    """Reference-reader table dump for (STAS, USGS)."""
    from golden_io import load_params
    return load_params("USGS", "STAS")
