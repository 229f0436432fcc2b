"""Fixture loading and comparison helpers shared by the CPU and GPU tests."""
from __future__ import annotations

import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def load_params(veg: str = "USGS", soil: str = "STAS") -> dict:
    return load(f"params_ref_{veg}_{soil}.npz")


def single_names() -> list[str]:
    return sorted(os.path.basename(p)[7:-4] for p in glob.glob(os.path.join(GOLDEN, "single_*.npz")))


def bit_equal(a, b) -> np.ndarray:
    """Elementwise identical (NaN == NaN), per element."""
    a = np.asarray(a)
    b = np.asarray(b)
    return (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)


def close(got, exp, rtol, atol) -> np.ndarray:
    got = np.asarray(got, np.float64)
    exp = np.asarray(exp, np.float64)
    both_nan = np.isnan(got) & np.isnan(exp)
    return both_nan | (np.abs(got - exp) <= atol + rtol * np.abs(exp))


def column_mismatch(got, exp, rtol, atol, names=None):
    """(bad-column mask, per-field worst report) for SoA arrays (nfield, n)."""
    ok = close(got, exp, rtol, atol)
    bad_cols = ~ok.all(axis=0)
    rep = []
    for f in np.nonzero(~ok.all(axis=1))[0]:
        i = np.nonzero(~ok[f])[0]
        d = np.abs(np.asarray(got[f, i], np.float64) - np.asarray(exp[f, i], np.float64))
        j = i[np.nanargmax(d)] if np.isfinite(d).any() else i[0]
        rep.append(f"{names[f] if names else f}: {i.size} cols, worst col {j} "
                   f"got {got[f, j]!r} exp {exp[f, j]!r}")
    return bad_cols, rep


def as_ref_status(status) -> np.ndarray:
    """Engine status bits as the reference harness can observe them.

    The reference raises FIRE<=0 (module_noahmp_func.f90:1291) and ZLVL<=ZPD
    (:3414) with the same message "STOP in Noah-MP", so its harness
    (oracle/ref_harness.f90) records both as ST_STOP (128)."""
    s = np.asarray(status, np.int32).copy()
    hit = (s & (4 | 16)) != 0
    s[hit] = (s[hit] & ~(4 | 16)) | 128
    return s
