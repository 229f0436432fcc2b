"""Noah-MP lookup tables (GENPARMMP / SOILPARMMP / VEGPARMMP.TBL).

`Params.from_tbl(dir, soil_tag, veg_tag)` parses the tables with the engine's
native reader (nmp_read_tables, same block/tag semantics as the reference
readers core/module_noahmp_{gen,soil,veg}_param.f90).  `Params.builtin()` loads
the parameter set shipped with the package (data/*.json), produced by that
same reader from the reference tables and pinned against the reference
Fortran readers' own dump (tests/test_tables.py).
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os

import numpy as np

from . import lib as _lib

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def builtin_path(soil_tag: str = "STAS", veg_tag: str = "USGS") -> str:
    return os.path.join(DATA_DIR, f"noahmp_params_{veg_tag}_{soil_tag}.json")


class Params:
    def __init__(self, struct: _lib.NmpParams, soil_tag: str, veg_tag: str):
        self.struct = struct
        self.soil_tag = soil_tag
        self.veg_tag = veg_tag

    # ---- constructors -------------------------------------------------------
    @classmethod
    def from_tbl(cls, tbl_dir: str, soil_tag: str = "STAS", veg_tag: str = "USGS") -> "Params":
        lib = _lib.load()
        s = _lib.NmpParams()
        _lib.check(lib.nmp_read_tables(tbl_dir.encode(), soil_tag.encode(), veg_tag.encode(),
                                       C.byref(s)), f"nmp_read_tables({tbl_dir})")
        return cls(s, soil_tag, veg_tag)

    @classmethod
    def from_dict(cls, d: dict, soil_tag: str = "STAS", veg_tag: str = "USGS") -> "Params":
        s = _lib.NmpParams()
        for name, ctype in _lib._PARAM_LAYOUT:
            v = d[name]
            if hasattr(ctype, "_length_"):
                flat = np.asarray(v, dtype=np.float64).reshape(-1)
                arr = getattr(s, name)
                if hasattr(ctype._type_, "_length_"):  # 2-D
                    inner = ctype._type_._length_
                    for i in range(ctype._length_):
                        for j in range(inner):
                            arr[i][j] = flat[i * inner + j]
                else:
                    for i in range(ctype._length_):
                        arr[i] = int(flat[i]) if ctype._type_ is C.c_int32 else flat[i]
            else:
                setattr(s, name, int(v) if ctype is C.c_int32 else float(v))
        return cls(s, soil_tag, veg_tag)

    @classmethod
    def from_json(cls, path: str) -> "Params":
        with open(path) as f:
            d = json.load(f)
        tags = d.pop("_tags", {"soil": "STAS", "veg": "USGS"})
        for k, v in d.items():
            if isinstance(v, list):
                d[k] = np.array(_denan(v), dtype=np.float64)
            elif v is None:
                d[k] = float("nan")
        return cls.from_dict(d, tags["soil"], tags["veg"])

    @classmethod
    def builtin(cls, soil_tag: str = "STAS", veg_tag: str = "USGS") -> "Params":
        return cls.from_json(builtin_path(soil_tag, veg_tag))

    # ---- views --------------------------------------------------------------
    def as_dict(self) -> dict:
        out = {}
        for name, ctype in _lib._PARAM_LAYOUT:
            v = getattr(self.struct, name)
            if hasattr(ctype, "_length_"):
                dt = np.int32 if (ctype._type_ is C.c_int32) else np.float32
                out[name] = np.ctypeslib.as_array(v).astype(dt).copy()
            else:
                out[name] = v
        return out

    def to_json(self, path: str):
        d = {}
        for k, v in self.as_dict().items():
            if isinstance(v, np.ndarray):
                d[k] = _nan2none(v.tolist())
            else:
                d[k] = None if (isinstance(v, float) and math.isnan(v)) else v
        d["_tags"] = {"soil": self.soil_tag, "veg": self.veg_tag}
        with open(path, "w") as f:
            json.dump(d, f, separators=(",", ":"))


def _nan2none(x):
    if isinstance(x, list):
        return [_nan2none(v) for v in x]
    if isinstance(x, float) and math.isnan(x):
        return None
    return x


def _denan(x):
    if isinstance(x, list):
        return [_denan(v) for v in x]
    return float("nan") if x is None else x
