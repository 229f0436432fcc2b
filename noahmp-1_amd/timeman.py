"""Offline time manager: calendar position and solar geometry per step.

The reference parses a begin/end datetime and a step length
(offline/noahmp_config.py:96-103, run/case.nml:13-27) but has no time loop;
`noahmp_sflx` expects JULIAN (fractional day of year, 0 <= JULIAN < YEARLEN),
YEARLEN and COSZ as inputs (core/module_noahmp_func.f90:67,122-128).  This
module supplies them, deterministically, for the offline driver.
"""
from __future__ import annotations

import datetime as _dt
import math

import numpy as np


def yearlen(year: int) -> int:
    return 366 if (year % 4 == 0 and (year % 100 != 0 or year % 400 == 0)) else 365


def julian(t: _dt.datetime) -> float:
    """Fractional day of year, 0-based (00:00 Jan 1 -> 0.0)."""
    start = _dt.datetime(t.year, 1, 1)
    return (t - start).total_seconds() / 86400.0


def step_times(begin: _dt.datetime, end: _dt.datetime, dt_seconds: float):
    """Model times of each step's *end*, like an offline driver stepping begin -> end."""
    n = int(round((end - begin).total_seconds() / dt_seconds))
    return [begin + _dt.timedelta(seconds=dt_seconds * (i + 1)) for i in range(n)]


def solar_terms(jul: float, ylen: int):
    """The step's column-independent factors of cosz: (sin decl, cos decl,
    ha0), ha0 = 2 pi x the UTC fraction of the day.  The device form of cosz
    (nmp_forcing_from_ldasin_geo) takes these from the host."""
    decl = 0.409 * math.sin(2.0 * math.pi * (jul - 80.0) / ylen)
    hour_utc = (jul - math.floor(jul)) * 24.0
    return math.sin(decl), math.cos(decl), 2.0 * math.pi * (hour_utc / 24.0)


def cosz(lat_rad, lon_rad, jul: float, ylen: int, sincos_lat=None):
    """Cosine of the solar zenith angle (simple declination + hour angle):
    sin lat sin decl + (cos lat cos decl) cos((ha0 + lon) - pi), in double.
    sincos_lat: (np.sin(lat), np.cos(lat)) precomputed by a caller that
    evaluates many steps of the same columns (the same values)."""
    sd, cd, ha0 = solar_terms(jul, ylen)
    ha = ha0 + np.asarray(lon_rad) - math.pi
    if sincos_lat is None:
        lat = np.asarray(lat_rad)
        sincos_lat = (np.sin(lat), np.cos(lat))
    return sincos_lat[0] * sd + sincos_lat[1] * cd * np.cos(ha)
