"""Native TBL reader (csrc/tables.cpp) vs the reference Fortran readers.

params_ref_*.npz hold what core/module_noahmp_{gen,soil,veg}_param.f90 read
from the reference tables (dumped by oracle/ref_harness.f90)."""
import os

import numpy as np
import pytest

from golden_io import bit_equal, load_params
from noahmp_amd import params as P

TAGS = [("STAS", "USGS"), ("STAS-RUC", "USGS"), ("STAS", "MODIFIED_IGBP_MODIS_NOAH"),
        ("STAS-RUC", "MODIFIED_IGBP_MODIS_NOAH")]
REF_TBL = "/root/reference/tbl"


def _assert_same(got: dict, exp: dict):
    bad = []
    for k, v in exp.items():
        g = np.asarray(got[k]).reshape(np.shape(v))
        if not bit_equal(np.asarray(g, np.asarray(v).dtype), v).all():
            bad.append(k)
    assert not bad, bad


@pytest.mark.parametrize("soil,veg", TAGS)
def test_builtin_params_match_reference_reader(soil, veg):
    _assert_same(P.Params.builtin(soil, veg).as_dict(), load_params(veg, soil))


@pytest.mark.parametrize("soil,veg", TAGS)
def test_native_reader_on_reference_tables(engine_lib, soil, veg):
    if not os.path.isdir(REF_TBL):
        pytest.skip("reference tables absent (GPU box)")
    _assert_same(P.Params.from_tbl(REF_TBL, soil, veg).as_dict(), load_params(veg, soil))


def test_native_reader_syntax(engine_lib, tmp_path):
    """List-directed records, tags, '/' record ends, quotes, CRLF, missing blocks."""
    (tmp_path / "GENPARMMP.TBL").write_text(
        "junk\r\n&noahmp_general_parameters\r\nSLOPE_DATA = 0.1, 0.6 , 1.0\r\n"
        "CSOIL_DATA = 2.00E+6 / trailing\r\nZBOT_DATA = -8.0\r\nCZIL_DATA = 0.1\r\n/\r\n")
    (tmp_path / "SOILPARMMP.TBL").write_text(
        "&noahmp_soil_X_parameters\nBEXP = 99\n/\n"
        "Soil Parameters\nSTAS\n2,1 'BB DRYSMC'\n"
        "1, 2.79, 0.010, 1.89, 0.339, 0.236, 0.069, 1.07E-6, 0.1, 0.010, 0.92, 'SAND'\n"
        "2, 4.26, 0.028, 1.06, 0.421, 0.383, 0.047, 1.41E-5, 0.2, 0.028, 0.82, 'LOAMY SAND'\n")
    (tmp_path / "VEGPARMMP.TBL").write_text("nothing here\n")
    s = P._lib.NmpParams()
    rc = engine_lib.nmp_read_tables(str(tmp_path).encode(), b"STAS", b"USGS", P.C.byref(s))
    # VEGPARMMP has no USGS block -> table error, never a silent default
    assert rc == -2
    assert "table" in engine_lib.nmp_strerror(rc).decode().lower()
    rc = engine_lib.nmp_read_tables(str(tmp_path / "nope").encode(), b"STAS", b"USGS",
                                    P.C.byref(s))
    assert rc == -2
