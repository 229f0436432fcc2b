"""Column order for wave coherence.

The step kernel runs one column per lane and a wave as slowly as its slowest
lane, so the order in which columns are laid out in memory decides which
columns share a wave.  Every column is independent and reads and writes only
its own index, so any permutation gives bit-identical per-column results;
the order is a layout choice made once, when the column set is built (the
offline driver orders the land points of the grid this way, the bench its
synthetic set).

Keys, in lexicographic priority (`coherent_order(..., key=...)`):
  "lon"            solar time: 2-degree longitude bands (day/night and the
                   diurnal phase are then shared by a wave)
  "lon-type"       + vegetation type (canopy or not, the canopy's parameters)
  "lon-snow-type"  + snow-covered or not, then vegetation type
  "lon-snow-type-soil"  + soil type
A grid already in row-major lat/lon order is mostly coherent; a shuffled
column set (the bench's config #3) is the worst case.
"""
from __future__ import annotations

import numpy as np

from . import layout as L

KEYS = ("lon", "lon-type", "lon-snow-type", "lon-snow-type-soil")


def coherent_order(lon_rad: np.ndarray, static_i: np.ndarray, isnow: np.ndarray,
                   key: str = "lon-type", band_deg: float = 2.0) -> np.ndarray:
    """Permutation of the columns (stable within equal keys)."""
    band = np.floor(np.degrees(np.asarray(lon_rad, np.float64)) / band_deg).astype(np.int64)
    if key == "lon":
        return np.argsort(band, kind="stable")
    vt = np.asarray(static_i[L.STATIC_I.index("VEGTYP")])
    if key == "lon-type":
        return np.lexsort((vt, band))
    if key == "lon-snow-type":
        return np.lexsort((vt, np.asarray(isnow) < 0, band))
    if key == "lon-snow-type-soil":
        st = np.asarray(static_i[L.STATIC_I.index("SOILTYP")])
        return np.lexsort((st, vt, np.asarray(isnow) < 0, band))
    raise ValueError(f"unknown column order key {key!r} (one of {KEYS})")
