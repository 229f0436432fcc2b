"""numpy restatement of the device forcing generator (csrc/forcing.hip,
nmp_forcing_synth) -- test infrastructure: same hash, same draws, same double
arithmetic in the same order, rounded once to the output precision."""
from __future__ import annotations

import math

import numpy as np

from noahmp_amd import layout as L

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(h):
    h = h ^ (h >> np.uint64(30))
    h = h * np.uint64(0xBF58476D1CE4E5B9)
    h = h ^ (h >> np.uint64(27))
    h = h * np.uint64(0x94D049BB133111EB)
    return h ^ (h >> np.uint64(31))


def _u(key, draw):
    h = _mix64(key + np.uint64(draw) * np.uint64(0xF1357AEA2E62A9C5))
    return (h >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def _n(key, d):
    u1, u2 = 1.0 - _u(key, d), _u(key, d + 1)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)


def synth(clim, julian: float, yearlen: int, seed: int, step: int, first_col: int = 0,
          dtype=np.float32):
    """(NFORCING, n) forcing of one step from (NCLIM, n) climate records."""
    c = {k: np.asarray(clim[i], np.float64) for i, k in enumerate(L.CLIMATE)}
    n = c["LAT"].shape[0]
    with np.errstate(over="ignore"):
        key = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
               + np.uint64(step) * np.uint64(0xD1B54A32D192ED03)
               + (np.arange(n, dtype=np.uint64) + np.uint64(first_col))
               * np.uint64(0xAEF17502108EF2D9))
        pi = 3.141592653589793
        frac = julian - math.floor(julian)
        hour = np.fmod(frac * 24.0 + c["LON"] * (180.0 / pi) / 15.0 + 48.0, 24.0)
        t = c["T0"] + c["AMP"] * np.cos(2.0 * pi * (hour - 14.0) / 24.0) + 0.3 * _n(key, 0)
        decl = 0.409 * math.sin(2.0 * pi * (julian - 80.0) / float(yearlen))
        ha = 2.0 * pi * frac + c["LON"] - pi
        cz = np.sin(c["LAT"]) * math.sin(decl) + np.cos(c["LAT"]) * math.cos(decl) * np.cos(ha)
        cloud = 0.6 * _u(key, 2)
        soldn = np.where(cz > 0.0, cz, 0.0) * 1000.0 * (1.0 - 0.6 * cloud)
        lwdn = (0.72 + 0.2 * cloud) * 5.67e-8 * (t * t) * (t * t)
        e = c["RH"] * 611.2 * np.exp(17.67 * (t - 273.15) / (t - 29.65))
        q2 = 0.622 * e / (c["PRES"] - 0.378 * e)
        prcp = np.where(_u(key, 3) < c["WET"], -1.0e-3 * np.log(1.0 - _u(key, 4)), 0.0)
        f = np.empty((L.NFORCING, n), np.float64)
        F = L.FORCING.index
        f[F("SFCTMP")] = t
        f[F("SFCPRS")] = c["PRES"]
        f[F("PSFC")] = c["PRES"]
        f[F("UU")] = c["WIND_U"] + 0.7 * _n(key, 5)
        f[F("VV")] = c["WIND_V"] + 0.7 * _n(key, 7)
        f[F("Q2")] = q2
        f[F("SOLDN")] = soldn
        f[F("LWDN")] = lwdn
        f[F("PRCP")] = prcp
        f[F("COSZ")] = cz
        f[F("CO2AIR")] = 395.0e-6 * c["PRES"]
        f[F("O2AIR")] = 0.209 * c["PRES"]
    return f.astype(dtype)
