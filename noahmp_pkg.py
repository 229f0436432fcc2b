"""Import helper: the package lives in ``noahmp-1_amd/`` (a name Python cannot
import directly); register it as ``noahmp_amd``."""
from __future__ import annotations

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "noahmp-1_amd")


def load_package():
    if "noahmp_amd" in sys.modules:
        return sys.modules["noahmp_amd"]
    spec = importlib.util.spec_from_file_location(
        "noahmp_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["noahmp_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


load_package()
