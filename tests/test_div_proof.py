"""The short-division range proof (tools/div_proof.py) holds for the domain the
kernel checks (csrc/vege_domain.h, the one copy of its limits), and the host's
stomata parameter flag admits every shipped vegetation table."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_short_division_site_is_inside_the_exact_region():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "div_proof.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "sites inside the exact region" in r.stdout
    assert r.stdout.count("stomata:") >= 7, "stomata bisection sites missing from the proof"
    for s in ("CTR = ", "TR = ", "DTV = B / A", "bare: DTG = B / A"):
        assert s in r.stdout, f"{s} missing from the proof"


def test_shipped_vegetation_tables_inside_the_stomata_box():
    """Every type of the four shipped table sets lies in the parameter box
    (otherwise its columns would run the bisection on IEEE division: correct,
    but not the measured path)."""
    import re
    import numpy as np
    sys.path.insert(0, ROOT)
    import noahmp_pkg  # noqa: F401
    from noahmp_amd.params import Params
    hdr = open(os.path.join(ROOT, "noahmp-1_amd", "csrc", "vege_domain.h")).read()
    D = {m.group(1): float(m.group(2))
         for m in re.finditer(r"#define NMP_DOM_(\w+) ([-+0-9.eE]+)", hdr)}
    for veg, soil in (("USGS", "STAS"), ("USGS", "STAS-RUC"),
                      ("MODIFIED_IGBP_MODIS_NOAH", "STAS"), ("MODIFIED_IGBP_MODIS_NOAH", "STAS-RUC")):
        p = Params.builtin(soil, veg).as_dict()

        def inside(k, name, zero_ok=False):
            v = np.asarray(p[k], np.float32)
            lo, hi = np.float32(D[name + "_LO"]), np.float32(D[name + "_HI"])
            ok = (v >= lo) & (v <= hi)
            return ok | (v == 0) if zero_ok else ok
        ok = (inside("kc25", "KC25") & inside("akc", "AKC") & inside("ko25", "KO25")
              & inside("ako", "AKO") & inside("avcmx", "AVCMX") & inside("mp", "MP")
              & inside("bp", "BP") & inside("qe25", "QE25", True)
              & ((np.asarray(p["vcmx25"]) == 0) | (inside("vcmx25", "VCMX25")
                                                    & inside("tmin", "TMIN"))))
        n = int(np.asarray(p["nlutyp"]).ravel()[0])   # the table's types (the rest is padding)
        assert n >= 20 and ok[:n].all(), (veg, soil, np.nonzero(~ok[:n])[0])
