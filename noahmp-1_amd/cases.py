"""Seeded synthetic column sets and forcing.

The reference's case files (forcing `ldasin/`, static `geo_em.d01.nc`,
`init.nc`; run/case.nml:2-11) are not shipped, so every benchmark and parity
input is generated here from ``numpy.random.Generator(PCG64(seed))``.  The
same generator feeds the GPU engine, the CPU oracles and the golden fixtures.

Kinds
  casenml  -- the single run/case.nml column (40N grassland on loam, USGS 7 /
              STAS 6), optionally replicated (BASELINE config #1/#2)
  mixed    -- vegetated USGS types, STAS soils 1-12, ISNOW uniform in
              {0,-1,-2,-3} with consistent snow layers (config #3)
  conus    -- all 27 USGS types / 19 soil types incl. water (IST=2), land
              ice (ICE=1), urban and barren (config #4)
All arrays are field-major SoA: (nfield, ncol).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import layout as L
from . import timeman

TFRZ = 273.15
CASE_NML_ZSOIL = np.array([-0.1, -0.4, -1.0, -2.0], dtype=np.float32)
VEGETATED_USGS = np.array([2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 17, 18, 20, 21, 22, 23])


@dataclass
class ColumnSet:
    static_f: np.ndarray  # (6, n) float32
    static_i: np.ndarray  # (6, n) int32
    state: np.ndarray     # (56, n) float32
    isnow: np.ndarray     # (n,) int32
    lon: np.ndarray       # (n,) radians (forcing generation only; not an sflx input)
    t0: np.ndarray        # (n,) mean air temperature of the column's climate
    amp: np.ndarray       # (n,) diurnal amplitude
    rh: np.ndarray        # (n,) relative humidity
    pres: np.ndarray      # (n,) surface pressure (Pa)
    wind: np.ndarray      # (2, n) mean wind
    wet: np.ndarray       # (n,) precipitation probability per step

    @property
    def n(self) -> int:
        return self.isnow.shape[0]

    def take(self, idx) -> "ColumnSet":
        return ColumnSet(*(a[..., idx] for a in (
            self.static_f, self.static_i, self.state, self.isnow, self.lon, self.t0, self.amp,
            self.rh, self.pres, self.wind, self.wet)))


def _esat(t):
    return 611.2 * np.exp(17.67 * (t - TFRZ) / (t - 29.65))


def _month_interp(table12, julian, lat):
    """LAI/SAI month interpolation like phenology (func.f90:578-598); table12 is (n, 12)."""
    day = np.where(lat >= 0, julian, np.mod(julian + 0.5 * 365.0, 365.0))
    t = 12.0 * day / 365.0
    it1 = np.floor(t + 0.5).astype(int)
    wt1 = (it1 + 0.5) - t
    it2 = it1 + 1
    it1 = np.where(it1 < 1, 12, it1)
    it2 = np.where(it2 > 12, 1, it2)
    rows = np.arange(table12.shape[0])
    return wt1 * table12[rows, it1 - 1] + (1.0 - wt1) * table12[rows, it2 - 1]


def make_columns(n: int, kind: str, params: dict, seed: int = 0, julian: float = 180.0,
                 zsoil=CASE_NML_ZSOIL, first: int = 0) -> ColumnSet:
    """Synthetic column set.  `first`: index of the first grid cell (kind "global",
    so the shards of a multi-GPU run tile the grid)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    zsoil = np.asarray(zsoil, dtype=np.float64)
    sf = np.zeros((L.NSTATIC_F, n), np.float64)
    si = np.zeros((L.NSTATIC_I, n), np.int32)
    st = np.zeros((L.NSTATE, n), np.float64)
    isnow = np.zeros(n, np.int32)

    iswater, isice, isurban, isbarren = (params[k] for k in ("iswater", "isice", "isurban",
                                                              "isbarren"))
    if kind == "casenml":
        lut = np.full(n, 7)
        slt = np.full(n, 6)
        isc = np.full(n, 4)
        slope = np.full(n, 1)
        lat = np.full(n, math.radians(40.0))
        lon = np.full(n, math.radians(-100.0))
        sf[L.STATIC_F.index("SHDFAC")] = 0.7
        sf[L.STATIC_F.index("SHDMAX")] = 0.8
        sf[L.STATIC_F.index("TBOT")] = 285.0
        t0 = np.full(n, 290.0)
        amp = np.full(n, 6.0)
        rh = np.full(n, 0.6)
        pres = np.full(n, 100000.0)
        wind = np.stack([np.full(n, 3.0), np.full(n, 1.0)])
        wet = np.full(n, 0.05)
    elif kind in ("mixed", "conus"):
        if kind == "mixed":
            lut = rng.choice(VEGETATED_USGS, n)
            slt = rng.integers(1, 13, n)
        else:
            lut = rng.integers(1, params["nlutyp"] + 1, n)
            land_soils = np.array([s for s in range(1, params["nsltyp"] + 1) if s != 14])
            slt = rng.choice(land_soils, n)
            slt = np.where(lut == iswater, 14, slt)
            slt = np.where(lut == isice, 16, slt)
        isc = rng.integers(1, 9, n)
        slope = rng.integers(1, 10, n)
        lat = np.radians(rng.uniform(-55.0, 70.0, n))
        lon = np.radians(rng.uniform(-180.0, 180.0, n))
        shd = rng.uniform(0.05, 0.95, n)
        sf[L.STATIC_F.index("SHDFAC")] = shd
        sf[L.STATIC_F.index("SHDMAX")] = np.minimum(1.0, shd + rng.uniform(0.0, 0.2, n))
        sf[L.STATIC_F.index("TBOT")] = rng.uniform(268.0, 300.0, n)
        t0 = rng.uniform(262.0, 292.0, n)     # straddles TFRZ
        amp = rng.uniform(2.0, 9.0, n)
        rh = rng.uniform(0.35, 0.95, n)
        pres = rng.uniform(85000.0, 102000.0, n)
        wind = rng.normal(0.0, 3.5, (2, n))
        wet = rng.uniform(0.0, 0.3, n)
    elif kind == "global":
        # config #5: the 0.25-degree global grid (1440 x 720), row-major from the
        # south-west corner; surface types drawn per 2-degree block (8 x 8 cells)
        # so neighbouring columns share them, as on a real grid; climate by latitude
        idx = (np.arange(n) + first) % (1440 * 720)
        row, col = idx // 1440, idx % 1440
        lat = np.radians(-89.875 + 0.25 * (row % 720))
        lon = np.radians(-179.875 + 0.25 * col)
        blk = (row // 8) * 180 + col // 8
        nblk = int(blk.max()) + 1
        blut = rng.integers(1, params["nlutyp"] + 1, nblk)
        land_soils = np.array([s for s in range(1, params["nsltyp"] + 1) if s != 14])
        bslt = rng.choice(land_soils, nblk)
        lut = blut[blk]
        alat = np.abs(np.degrees(lat))
        lut = np.where(alat > 66.0, np.where((blk % 3) == 0, isice, lut), lut)
        slt = np.where(lut == iswater, 14, np.where(lut == isice, 16, bslt[blk]))
        isc = rng.integers(1, 9, nblk)[blk]
        slope = rng.integers(1, 10, nblk)[blk]
        shd = rng.uniform(0.05, 0.95, nblk)[blk]
        sf[L.STATIC_F.index("SHDFAC")] = shd
        sf[L.STATIC_F.index("SHDMAX")] = np.minimum(1.0, shd + rng.uniform(0.0, 0.2, n))
        t0 = 301.0 - 45.0 * np.abs(np.sin(lat)) ** 1.5 + rng.normal(0.0, 1.5, n)
        sf[L.STATIC_F.index("TBOT")] = t0 - 3.0 + rng.uniform(-1.0, 1.0, n)
        amp = rng.uniform(2.0, 9.0, n)
        rh = rng.uniform(0.35, 0.95, n)
        pres = rng.uniform(85000.0, 102000.0, n)
        wind = rng.normal(0.0, 3.5, (2, n))
        wet = rng.uniform(0.0, 0.3, n)
    else:
        raise ValueError(f"unknown column kind {kind!r}")

    sf[L.STATIC_F.index("LAT")] = lat
    sf[L.STATIC_F.index("ZLVL")] = 10.0
    sf[L.STATIC_F.index("FOLN")] = 1.0
    si[L.STATIC_I.index("VEGTYP")] = lut
    si[L.STATIC_I.index("SOILTYP")] = slt
    si[L.STATIC_I.index("SLOPETYP")] = slope
    si[L.STATIC_I.index("SOILCOLOR")] = isc
    ist = np.where(lut == iswater, 2, 1)
    si[L.STATIC_I.index("IST")] = ist
    si[L.STATIC_I.index("ICE")] = np.where(lut == isice, 1, 0)

    smcmax = np.asarray(params["smcmax"])[slt - 1]
    smcwlt = np.asarray(params["smcwlt"])[slt - 1]

    # ---- snow --------------------------------------------------------------
    if kind == "casenml":
        isnow[:] = 0
    else:
        isnow[:] = rng.choice(np.array([0, -1, -2, -3]), n)
        cold = t0 < 276.0
        isnow[:] = np.where(cold | (lut == isice), isnow, 0)
        isnow[:] = np.where(ist == 2, 0, isnow)
    stc = np.zeros((7, n))
    snice = np.zeros((3, n))
    snliq = np.zeros((3, n))
    dzs = np.zeros((3, n))
    dz_lo = np.array([0.02, 0.05, 0.10])
    dz_hi = np.array([0.05, 0.20, 0.40])
    for j in range(3):                       # C index j <-> Fortran layer j-2
        m = j - 2 > isnow                     # active: layer index >= isnow+1
        pos = j - (3 + isnow)                 # 0 = top active layer
        lo = dz_lo[np.clip(pos, 0, 2)]
        hi = dz_hi[np.clip(pos, 0, 2)]
        dz = rng.uniform(lo, hi)
        rho = rng.uniform(80.0, 350.0, n)
        dzs[j] = np.where(m, dz, 0.0)
        snice[j] = np.where(m, dz * rho, 0.0)
        snliq[j] = np.where(m, snice[j] * rng.uniform(0.0, 0.05, n), 0.0)
        stc[j] = np.where(m, rng.uniform(252.0, TFRZ - 0.05, n), 0.0)
    snowh = dzs.sum(0)
    sneqv = (snice + snliq).sum(0)
    thin = (isnow == 0) & (rng.uniform(size=n) < (0.0 if kind == "casenml" else 0.3)) & (t0 < 280)
    snowh = np.where(thin, rng.uniform(0.001, 0.02, n), snowh)
    sneqv = np.where(thin, snowh * rng.uniform(60.0, 250.0, n), sneqv)

    # ---- soil --------------------------------------------------------------
    if kind == "casenml":
        tsoil = np.stack([np.full(n, v) for v in (289.0, 288.0, 286.5, 285.5)])
    else:
        base = np.where(isnow < 0, rng.uniform(264.0, 276.0, n), rng.uniform(266.0, 300.0, n))
        tsoil = np.stack([base + rng.normal(0.0, 1.0, n) * (k + 1) * 0.6 for k in range(4)])
    stc[3:] = tsoil
    smc = np.stack([rng.uniform(smcwlt + 0.02, smcmax - 0.02) for _ in range(4)])
    if kind == "casenml":
        smc = np.stack([np.full(n, v) for v in (0.30, 0.29, 0.28, 0.28)])
    frozen = tsoil < TFRZ
    sh2o = np.where(frozen, smc * rng.uniform(0.1, 0.6, (4, n)), smc)
    smc = np.where(ist == 2, 1.0, smc)
    sh2o = np.where(ist == 2, 1.0, sh2o)

    zsnso = np.zeros((7, n))
    # snow layer bottoms (negative, from snow surface), then soil bottoms shifted by snowh
    acc = np.zeros(n)
    for j in range(3):
        m = j - 2 > isnow
        acc = acc - np.where(m, dzs[j], 0.0)
        zsnso[j] = np.where(m, acc, 0.0)
    layered_h = np.where(isnow < 0, snowh, 0.0)
    for k in range(4):
        zsnso[3 + k] = zsoil[k] - layered_h

    # ---- canopy / air ----------------------------------------------------------
    ta = t0 + rng.normal(0.0, 1.0, n)
    tv = ta + rng.uniform(-1.5, 1.5, n)
    top = np.where(isnow < 0, stc[np.clip(3 + isnow, 0, 2), np.arange(n)], tsoil[0])
    tg = np.where(isnow < 0, np.minimum(top, TFRZ), tsoil[0])
    eah = rh * _esat(ta) * rng.uniform(0.9, 1.0, n)
    q2 = 0.622 * eah / (pres - 0.378 * eah)
    fwet = rng.uniform(0.0, 0.4, n)
    canliq = np.where(tv > TFRZ, rng.uniform(0.0, 0.2, n), 0.0)
    canice = np.where(tv <= TFRZ, rng.uniform(0.0, 0.2, n), 0.0)

    # ---- groundwater (HRLDAS-style init, groundwater() :6580) -----------------
    zwt = rng.uniform(2.2, 6.0, n)
    shallow = rng.uniform(size=n) < (0.0 if kind == "casenml" else 0.2)
    zwt = np.where(shallow, rng.uniform(1.5, 1.95, n), zwt)
    if kind == "casenml":
        zwt[:] = 2.5
    wa = (-zsoil[3] + 25.0 - zwt) * 1000.0 * 0.2
    wa = np.where(shallow, 5000.0, wa)
    wt = wa + np.where(shallow, (2.0 - zwt) * 1000.0 * 0.25, 0.0)

    # ---- vegetation / carbon -----------------------------------------------------
    lai12 = np.asarray(params["lai12m"])[lut - 1]
    sai12 = np.asarray(params["sai12m"])[lut - 1]
    lai = _month_interp(lai12, julian, lat)
    sai = _month_interp(sai12, julian, lat)
    sla = np.asarray(params["sla"])[lut - 1]
    lfmass = np.where(sla > 0, lai * 1000.0 / np.maximum(sla, 1e-6), 0.0)
    stmass = sai / 0.003
    wdpool = np.asarray(params["wdpool"])[lut - 1]

    S = L.si
    st[L.s("STC")] = stc
    st[L.s("ZSNSO")] = zsnso
    st[L.s("SNICE")] = snice
    st[L.s("SNLIQ")] = snliq
    st[L.s("SH2O")] = sh2o
    st[L.s("SMC")] = smc
    st[S("TV")] = tv
    st[S("TG")] = tg
    st[S("TAH")] = ta
    st[S("EAH")] = eah
    st[S("FWET")] = fwet
    st[S("CANLIQ")] = canliq
    st[S("CANICE")] = canice
    st[S("QSFC")] = q2
    st[S("SNOWH")] = snowh
    st[S("SNEQV")] = sneqv
    st[S("SNEQVO")] = sneqv * rng.uniform(0.95, 1.0, n)
    st[S("ALBOLD")] = rng.uniform(0.5, 0.85, n)
    st[S("TAUSS")] = np.where(sneqv > 0, rng.uniform(0.0, 2.0, n), 0.0)
    st[S("QSNOW")] = np.where(rng.uniform(size=n) < 0.2, rng.uniform(0.0, 5e-4, n), 0.0)
    st[S("ZWT")] = zwt
    st[S("WA")] = wa
    st[S("WT")] = wt
    st[S("WSLAKE")] = 0.0
    st[S("LAI")] = lai
    st[S("SAI")] = sai
    st[S("LFMASS")] = lfmass
    st[S("RTMASS")] = rng.uniform(300.0, 700.0, n)
    st[S("STMASS")] = stmass
    st[S("WOOD")] = rng.uniform(0.0, 1000.0, n) * wdpool
    st[S("STBLCP")] = rng.uniform(500.0, 2000.0, n)
    st[S("FASTCP")] = rng.uniform(500.0, 2000.0, n)
    st[S("CM")] = rng.uniform(0.002, 0.02, n)
    st[S("CH")] = rng.uniform(0.002, 0.02, n)

    return ColumnSet(sf.astype(np.float32), si, st.astype(np.float32), isnow, lon, t0, amp, rh,
                     pres, wind, wet)


def forcing_step(cols: ColumnSet, julian: float, ylen: int, step: int, seed: int = 0,
                 dtype=np.float32) -> np.ndarray:
    """Deterministic per-column diurnal forcing for one step, shape (12, n).

    SFCTMP = T0 + A cos(2 pi (h_local - 14)/24); COSZ from lat/lon/date;
    SOLDN = S0 cos(z)+; LWDN from an effective sky emissivity; precipitation
    pulses with a per-column wet probability."""
    n = cols.n
    rng = np.random.Generator(np.random.PCG64((seed * 1_000_003 + step) & 0xFFFFFFFF))
    lat = cols.static_f[L.STATIC_F.index("LAT")].astype(np.float64)
    hour_local = ((julian - math.floor(julian)) * 24.0 + np.degrees(cols.lon) / 15.0) % 24.0
    t = cols.t0 + cols.amp * np.cos(2.0 * math.pi * (hour_local - 14.0) / 24.0)
    t = t + rng.normal(0.0, 0.3, n)
    cz = timeman.cosz(lat, cols.lon, julian, ylen)
    cloud = rng.uniform(0.0, 0.6, n)
    soldn = np.maximum(cz, 0.0) * 1000.0 * (1.0 - 0.6 * cloud)
    eps_a = 0.72 + 0.2 * cloud
    lwdn = eps_a * 5.67e-8 * t ** 4
    e = cols.rh * _esat(t)
    q2 = 0.622 * e / (cols.pres - 0.378 * e)
    rain = rng.uniform(size=n) < cols.wet
    prcp = np.where(rain, rng.exponential(1.0e-3, n), 0.0)
    f = np.empty((L.NFORCING, n), np.float64)
    F = L.FORCING.index
    f[F("SFCTMP")] = t
    f[F("SFCPRS")] = cols.pres
    f[F("PSFC")] = cols.pres
    f[F("UU")] = cols.wind[0] + rng.normal(0.0, 0.7, n)
    f[F("VV")] = cols.wind[1] + rng.normal(0.0, 0.7, n)
    f[F("Q2")] = q2
    f[F("SOLDN")] = soldn
    f[F("LWDN")] = lwdn
    f[F("PRCP")] = prcp
    f[F("COSZ")] = cz
    f[F("CO2AIR")] = 395.0e-6 * cols.pres
    f[F("O2AIR")] = 0.209 * cols.pres
    return f.astype(dtype)


def forcing_random(cols: ColumnSet, seed: int = 0) -> np.ndarray:
    """Independent per-column forcing for single-call parity sets: covers day
    and night (COSZ <= 0), rain, snow, calm and windy cases in one step."""
    n = cols.n
    rng = np.random.Generator(np.random.PCG64(seed + 7919))
    t = cols.t0 + rng.uniform(-1.0, 1.0, n) * cols.amp
    cz = rng.uniform(-0.6, 1.0, n)
    soldn = np.where(cz > 0, rng.uniform(0.0, 1000.0, n) * np.maximum(cz, 0.0), 0.0)
    lwdn = rng.uniform(0.65, 0.95, n) * 5.67e-8 * t ** 4
    e = cols.rh * _esat(t)
    q2 = 0.622 * e / (cols.pres - 0.378 * e)
    prcp = np.where(rng.uniform(size=n) < 0.35, rng.exponential(1.5e-3, n), 0.0)
    f = np.empty((L.NFORCING, n), np.float64)
    F = L.FORCING.index
    f[F("SFCTMP")] = t
    f[F("SFCPRS")] = cols.pres
    f[F("PSFC")] = cols.pres * rng.uniform(0.995, 1.0, n)
    f[F("UU")] = rng.normal(0.0, 4.0, n)
    f[F("VV")] = rng.normal(0.0, 4.0, n)
    f[F("Q2")] = q2
    f[F("SOLDN")] = soldn
    f[F("LWDN")] = lwdn
    f[F("PRCP")] = prcp
    f[F("COSZ")] = cz
    f[F("CO2AIR")] = 395.0e-6 * cols.pres
    f[F("O2AIR")] = 0.209 * cols.pres
    return f.astype(np.float32)


def climate(cols: ColumnSet, dtype=np.float64) -> np.ndarray:
    """(NCLIM, n) climate records for the device forcing generator
    (nmp_forcing_synth, layout.CLIMATE): the per-column parameters that
    forcing_step draws its diurnal cycle from."""
    c = np.empty((L.NCLIM, cols.n), np.float64)
    c[L.CLIMATE.index("LAT")] = cols.static_f[L.STATIC_F.index("LAT")]
    c[L.CLIMATE.index("LON")] = cols.lon
    c[L.CLIMATE.index("T0")] = cols.t0
    c[L.CLIMATE.index("AMP")] = cols.amp
    c[L.CLIMATE.index("RH")] = cols.rh
    c[L.CLIMATE.index("PRES")] = cols.pres
    c[L.CLIMATE.index("WIND_U")] = cols.wind[0]
    c[L.CLIMATE.index("WIND_V")] = cols.wind[1]
    c[L.CLIMATE.index("WET")] = cols.wet
    return c.astype(dtype)
