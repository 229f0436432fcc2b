"""Regenerate noahmp-1_amd/data/noahmp_params_<VEG>_<SOIL>.json from TBL files
with the engine's own reader (nmp_read_tables).

usage: python tools/make_params.py [TBL_DIR]   (default: /root/reference/tbl)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import noahmp_pkg  # noqa: E402,F401
from noahmp_amd import params  # noqa: E402

TAGS = [("STAS", "USGS"), ("STAS-RUC", "USGS"), ("STAS", "MODIFIED_IGBP_MODIS_NOAH"),
        ("STAS-RUC", "MODIFIED_IGBP_MODIS_NOAH")]

if __name__ == "__main__":
    tbl = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/tbl"
    os.makedirs(params.DATA_DIR, exist_ok=True)
    for soil, veg in TAGS:
        p = params.Params.from_tbl(tbl, soil, veg)
        out = params.builtin_path(soil, veg)
        p.to_json(out)
        print("wrote", out)
