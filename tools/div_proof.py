"""Range proof of the short divisions (DivFast32) in the canopy and bare-ground
Newton loops, the stomata bisection and the soil-water sub-steps.

DivFast32 (csrc/sflx_math.h) returns IEEE a/b bit for bit when
  b is normal with a normal reciprocal: |b| in [2^-126, 2^126],
  the fma residual a - b*q is not subnormal: a = 0 or |a| >= 2^-102,
  the quotient is normal: a = 0 or |a/b| in [2^-126, 2^126],
or when an operand is zero, infinite or NaN (v_div_fixup_f32 takes over).
The first three hold on every pair of significands at every scale
(tools/fdiv_exhaust.hip, profiles/r03/fdiv_exhaust2.txt).

This script derives, for every division the loop runs with DivFast32, a
bound on |a|, |b| and |a/b| from the input domain of csrc/vege_domain.h (the
kernel checks it per column and falls back to IEEE division outside it), in
the loop's own order (sflx_kernel.hip vege_flux; func.f90:2744-2877 with
sfcdif1 :3353-3508 and ragrb :3260-3350), and checks each against that
region.  Magnitudes are intervals [lo, hi] of |x| for nonzero x plus a flag
for "x may be 0".  Every bound is widened by 2^-20 per operation, more than
the kernel's rounding (2^-24 per operation, a few ulps per libm call).

Differences of floats are bounded below by granularity: x - y (x, y floats)
is 0 or at least 2^(E - 23), E the smaller binary exponent of x and y,
because both are multiples of that power of two; rounding keeps it.

Loop-carried values are bounded by induction over the iterations: the values
an iteration starts from (TV, TAH, H, HG, FV, FHG, MOZ/FM/FH) are assumed in
the intervals below, the iteration is shown to end inside them again; TV and
RAHG are the two the kernel checks at run time, every iteration.

    python tools/div_proof.py            # prints the per-site table, exit 1 on a failure
"""
import math
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "noahmp-1_amd", "csrc", "vege_domain.h")

W = 2.0 ** -20            # widening per operation
A_MIN = 2.0 ** -102       # smallest nonzero numerator
N_MIN, N_MAX = 2.0 ** -126, 2.0 ** 126
KARMAN, GRAV, CPAIR, SB = 0.4, 9.80616, 1004.64, 5.67e-08
HVAP, HSUB, TFRZ = 2.51e6, 2.8440e6, 273.16


def domain():
    d = {}
    for m in re.finditer(r"#define (NMP_DOM_\w+) ([-+0-9.eE]+)", open(HDR).read()):
        d[m.group(1)[8:]] = float(m.group(2))
    return d


class M:
    """|x| in [lo, hi] for x != 0; z: x may be 0."""

    def __init__(self, lo, hi, z=False):
        assert 0 < lo <= hi, (lo, hi)
        self.lo, self.hi, self.z = lo * (1 - W), hi * (1 + W), z

    def __mul__(self, o):
        o = o if isinstance(o, M) else M(abs(o), abs(o))
        return M(self.lo * o.lo, self.hi * o.hi, self.z or o.z)

    __rmul__ = __mul__

    def __add__(self, o):   # terms of one sign (all >= 0 here)
        lo = min(self.lo, o.lo) if (self.z or o.z) else max(self.lo, o.lo)
        return M(lo, self.hi + o.hi, self.z and o.z)

    def nz(self):           # the same magnitudes, known nonzero
        return M(self.lo, self.hi)

    def __repr__(self):
        return f"{'0|' if self.z else ''}[{self.lo:.3g}, {self.hi:.3g}]"


def c(v):
    return M(abs(v), abs(v))


def diff(x, y):
    """|x - y| for floats x, y with |x| <= x.hi etc.: 0 or >= 2^(E-23)."""
    e = math.floor(math.log2(min(x.lo, y.lo)))
    return M(2.0 ** (e - 23), x.hi + y.hi, True)


def fn(f, x):            # monotone increasing f on magnitudes
    return M(f(x.lo), f(x.hi), x.z)


rows, bad = [], []


def site(name, a, b, ref, note=""):
    """Record one division a/b; returns the quotient's magnitude interval."""
    q = M(a.lo / b.hi, a.hi / b.lo, a.z)
    ok = (not b.z and N_MIN <= b.lo and b.hi <= N_MAX and A_MIN <= a.lo
          and N_MIN <= q.lo and q.hi <= N_MAX)
    rows.append((name, ref, a, b, q, ok, note))
    if not ok:
        bad.append(name)
    return q


def sqrt_site(name, x, ref, note=""):
    """sqrt_normal32 (csrc/sflx_math.h) equals IEEE sqrtf for finite x >= 2^-96:
    the IEEE lowering's own instructions minus its scaling of smaller x and
    its zero / infinity / NaN select."""
    ok = not x.z and 2.0 ** -96 <= x.lo and x.hi <= 3.4028234e38
    rows.append((name, ref, x, M(1.0, 1.0), fn(math.sqrt, x), ok,
                 ("sqrt: " + note) if note else "sqrt"))
    if not ok:
        bad.append(name)


def esat_range():
    def poly(t, cs):
        v = 0.0
        for k in reversed(cs):
            v = v * t + k
        return 100.0 * v
    w = [6.107799961, 4.436518521E-01, 1.428945805E-02, 2.650648471E-04, 3.031240396E-06,
         2.034080948E-08, 6.136820929E-11]
    i = [6.109177956, 5.034698970E-01, 1.886013408E-02, 4.176223716E-04, 5.824720280E-06,
         4.838803174E-08, 1.838826904E-10]
    dw = [4.438099984E-01, 2.857002636E-02, 7.938054040E-04, 1.215215065E-05, 1.036561403E-07,
          3.532421810e-10, -7.090244804E-13]
    di = [5.030305237E-01, 3.773255020E-02, 1.267995369E-03, 2.477563108E-05, 3.005693132E-07,
          2.158542548E-09, 7.131097725E-12]
    ts = [k / 100.0 for k in range(-5000, 5001)]   # tdc clamps to [-50, 50] C
    es = [poly(t, w if t > 0 else i) for t in ts]
    des = [poly(t, dw if t > 0 else di) for t in ts]
    return M(min(es), max(es)), M(min(des), max(des))


def stomata_sites(D, T, p, es, rb):
    """The stomata bisection's divisions (func.f90:3850-3879; sflx_kernel.hip
    stomata_solve), per 1 K band of the canopy temperature TV: KC, KO, CP, AWC
    and VCMX are functions of TV, so bounding them band by band keeps their
    correlation (a hot canopy has a large KC and a small VCMX together).  Each
    site's row is the worst case over the bands."""
    RGAS, MPE = 8.314, 1e-6
    box = lambda k: (D[k + "_LO"], D[k + "_HI"])
    kc25, akc, ko25, ako, avcmx = box("KC25"), box("AKC"), box("KO25"), box("AKO"), box("AVCMX")
    vcmx25, qe25, mp, bp = box("VCMX25"), box("QE25"), box("MP"), box("BP")
    co2, o2 = M(*box("CO2")), M(*box("O2"))
    apar, eah = M(*box("APAR")), M(D["EAH_LO"], D["EAH_HI"], True)
    fnf = M(D["FNF_LO"], 1.0, True)
    btran = M(MPE, 1.0001)                        # MAX(MPE, sum of root-layer shares)
    cf = M(p.lo / (RGAS * T.hi) * 1e6, p.hi / (RGAS * T.lo) * 1e6)
    rlb = M(rb.lo / cf.hi, rb.hi / cf.lo)         # RLB = RB / CF (IEEE, stomata_pre)
    worst = {}

    def pw(base, ex0, ex1):                       # base**ex over a box of bases and exponents
        vals = [b ** e for b in base for e in (ex0, ex1)]
        return min(vals), max(vals)

    def g(t):                                      # the VCMX temperature factor's exponent
        return (-2.2e5 + 710.0 * t) / (8.314 * t)

    t_hi = D["STOMATA_TV_HI"]                    # checked before the calls
    t0 = T.lo
    while t0 < t_hi:
        t1 = min(t0 + 1.0, t_hi)
        ex0, ex1 = (t0 - TFRZ - 25.0) / 10.0, (t1 - TFRZ - 25.0) / 10.0
        a_lo, a_hi = pw(akc, ex0, ex1)
        kc = M(kc25[0] * a_lo, kc25[1] * a_hi)
        o_lo, o_hi = pw(ako, ex0, ex1)
        ko = M(ko25[0] * o_lo, ko25[1] * o_hi)
        awc = M(kc.lo * (1 + o2.lo / ko.hi), kc.hi * (1 + o2.hi / ko.lo))
        cp = M(0.105 * kc.lo * o2.lo / ko.hi, 0.105 * kc.hi * o2.hi / ko.lo)
        v_lo, v_hi = pw(avcmx, ex0, ex1)
        efac = M(1 + math.exp(g(t0)), 1 + math.exp(g(t1)))
        vcmx = M(vcmx25[0] / efac.hi * fnf.lo * btran.lo * v_lo,
                 vcmx25[1] / efac.lo * 1.0 * btran.hi * v_hi, True)
        j = M(4.6 * apar.lo * qe25[0], 4.6 * apar.hi * qe25[1], True)
        ci = M(1.5 * co2.lo * 2.0 ** -20, 1.5 * co2.hi)   # bisection midpoints of [0, 1.5 CO2]
        dci = diff(ci, cp)                        # MAX(CI - CP, 0): 0 or >= granularity
        rows_before = len(rows)
        wj = site("stomata: WJ = (CI-CP)*J / (CI+2CP)", dci * j,
                  M(ci.lo + 2 * cp.lo, ci.hi + 2 * cp.hi), ":3860")
        wc = site("stomata: WC = (CI-CP)*VCMX / (CI+AWC)", dci * vcmx,
                  M(ci.lo + awc.lo, ci.hi + awc.hi), ":3861")
        we4 = site("stomata: WE = 4000*VCMX*CI / SFCPRS (C4)", 4000 * vcmx * ci, p, ":3866")
        we3 = 0.5 * vcmx
        lo = min(wj.lo, wc.lo, min(we3.lo, we4.lo))
        # PSN = MIN(WJ, WC, WE) * IGS (IGS = 0 or 1) <= MIN(J, VCMX): WJ <= J and
        # WC <= VCMX because (CI-CP) < CI+2CP and < CI+AWC (C3); WJ = J, WC =
        # VCMX (C4) -- a bound interval arithmetic on the quotients loses
        hi = min(j.hi, vcmx.hi)
        psn = M(lo, hi, True)
        cs = M(MPE, co2.hi)                       # MAX(CO2 - 1.37 RLB SFCPRS PSN, MPE)
        num = M(mp[0], mp[1]) * psn * p
        if t1 > D["TMIN_LO"]:
            x = site("stomata: A = MP*PSN*SFCPRS*EA / (CS*EI)", num * eah, cs * es, ":3870",
                     "EA = EAH, EI = ESTV; PSN > 0 needs TV > TMIN >= TMIN_LO")
            xb = site("stomata: B = MP*PSN*SFCPRS / CS", num, cs, ":3871")
        else:                                     # PSN = 0 (IGS = 0 or VCMX25 = 0): a = 0
            x, xb = M(num.lo / cs.hi, num.hi / cs.lo), M(num.lo / cs.hi, num.hi / cs.lo)
        a = M(bp[0], x.hi + bp[1])
        bmag = M(1e-30, (xb.hi + bp[1]) * rlb.hi + 1.0, True)
        sqrt_site("stomata: SQRT(B*B - 4*A*C)", M(4 * a.lo * rlb.lo, bmag.hi ** 2 + 4 * a.hi * rlb.hi),
                  ":3873", "C = -RLB < 0, so the radicand is >= 4*A*RLB")
        q = M(math.sqrt(a.lo * rlb.lo), bmag.hi + math.sqrt(a.hi * rlb.hi))
        site("stomata: R1 = Q / A", q, a, ":3875")
        site("stomata: R2 = C / Q", rlb, q, ":3876", "C = -RLB")
        for r in rows[rows_before:]:
            name = r[0]
            if name not in worst or not r[5] or (worst[name][5] and r[4].lo < worst[name][4].lo):
                worst[name] = r
        del rows[rows_before:]
        t0 = t1
    global bad
    bad = [b for b in bad if not b.startswith("stomata:")]
    for name, r in worst.items():
        rows.append(r)
        if not r[5]:
            bad.append(name)


def soil_sites():
    """The soil-water sub-steps' divisions by the layer thicknesses (srt,
    func.f90:6238-6276; sflx_kernel.hip NMP_SOIL_DIV).  Their denominators are
    launch-uniform differences of ZSOIL, which the kernel checks once against
    [2^-20, 2^20] (outside: every such division on IEEE).  Their numerators
    (2, 2*(SMX(K)-SMX(K+1)), WDF*DDZ, WFLUX) are not bounded away from 0 --
    WDF of very dry clay is ~1e-32 -- so the kernel checks each numerator at
    run time: a = 0 or 2^-102 <= |a| <= 2^100, else that lane divides on IEEE.
    Inside both checks the quotient lies in [2^-122, 2^120]."""
    den = M(2.0 ** -20, 2.0 ** 20)
    num = M(A_MIN * (1 + 2 * W), 2.0 ** 100, True)  # (M widens its bounds by W)
    note = "numerator window checked per lane, IEEE outside"
    site("soil: DDZ = 2 / TEMP1", c(2.0), den, ":6243")
    site("soil: DSMDZ = 2*(SMX(K)-SMX(K+1)) / TEMP1", num, den, ":6244", note)
    site("soil: AI, CI, BI = -WDF*DDZ / DENOM", num, den, ":6266-6272", note)
    site("soil: RHSTT = WFLUX / (-DENOM)", num, den, ":6275", note)


def main():
    D = domain()
    # ---- loop-invariant inputs: the kernel's entry check (vege_domain.h) ----
    T = M(D["T_LO"], D["T_HI"])                    # SFCTMP, TG; TV (every iteration)
    rho = M(D["RHO_LO"], D["RHO_HI"])
    rhocp = rho * CPAIR
    qair = M(1e-30, 1.0, True)                     # checked 0 <= QAIR <= 1
    tvir = M(T.lo, T.hi * 1.61)                    # (1 + 0.61 QAIR) SFCTMP
    ur = M(1.0, D["UR_HI"])
    tmpc = M(D["TMPC_LO"], D["TMPC_HI"])           # TMPCM = TMPCH, TMPCM2 = TMPCH2
    dz = M(D["DZ_LO"], D["DZ_HI"])                 # ZLVL - ZPD
    z0 = M(D["Z0_LO"], D["Z0_HI"])                 # Z0M = Z0H, Z0MG
    d2 = M(2.0, 2.0 + D["Z0_HI"])                  # 2 + Z0H
    hcan = M(D["HCAN_LO"], D["HCAN_HI"])
    zpd = M(D["Z0_LO"], D["HCAN_HI"], True)        # 0 or >= Z0_LO, <= HCAN
    cwph = M(D["CWPH_LO"], D["CWPH_HI"])           # CWP * VAIE * HCAN
    vaie = M(D["VAI_LO"], 6.0)
    lai = M(D["LAI_LO"], 6.0, True)
    fwet = M(D["FWET_LO"], 1.0, True)
    fveg = M(D["FVEG_LO"], 1.0)
    sdl = M(D["SDL_LO"], D["SDL_HI"])              # SQRT(DLEAF/UC)
    rsurf_hi = D["RSURF_HI"]
    p = M(D["P_LO"], D["P_HI"])
    eair_hi = D["EAIR_HI"]
    gammav = M(CPAIR * p.lo / (0.622 * HSUB), CPAIR * p.hi / (0.622 * HVAP))
    es, des = esat_range()                          # ESTG, ESTV and DESTV
    rs_hi = D["RS_HI"]
    rahg_w = M(D["RAHG_LO"], D["RAHG_HI"])          # checked every iteration
    tah = M(T.lo * (1 - 1e-5), T.hi * (1 + 1e-5))   # convex combination of SFCTMP, TG, TV
    dT = diff(T, tah)                               # TAH - SFCTMP, TG - TAH, TV - TAH

    # ---- loop-carried values an iteration starts from (induction hypothesis) ----
    cmfm = M(0.1 * tmpc.lo, tmpc.hi + 5.0)          # TMPCM - FM, FM in [-5, 0.9 TMPCM]
    cm = M(0.16 / cmfm.hi ** 2, 0.16 / cmfm.lo ** 2)
    fv = ur * fn(math.sqrt, cm)                     # FV = UR * SQRT(CM)
    rahc = M(1.0, 1.0 / (cm.lo * ur.lo))            # MAX(1, 1/(CH*UR))
    h = M((rhocp * dT).lo / rahc.hi, (rhocp * dT).hi, True)
    hg = M((rhocp * dT).lo / rahg_w.hi, (rhocp * dT).hi / rahg_w.lo, True)
    fhg_lo = None                                   # derived below, then checked

    # ---- sfcdif1 (iter >= 2), :3405-3441, sflx_kernel.hip sfcdif1 ----
    kgtv = KARMAN * site("GRAV / TVIR", c(GRAV), tvir, ":3430 (once per loop)")
    tmp1 = site("TMP1 = KGTV*H / RHOCP", kgtv * h, rhocp, ":3431")
    tmp1 = M(1e-6, tmp1.hi)                         # IF (ABS(TMP1) <= MPE) TMP1 = MPE
    fv3 = fn(lambda x: x ** 3, fv)
    mol = site("MOL = -FV**3 / TMP1", fv3, tmp1, ":3433")
    site("MOZ = (ZLVL-ZPD) / MOL", dz, mol, ":3434", "then MIN(., 1)")
    site("MOZ2 = (2+Z0H) / MOL", d2, mol, ":3435", "then MIN(., 1)")
    cm_q = site("CM = KARMAN**2 / CMFM**2", c(0.16), cmfm * cmfm, ":3499",
                "CMFM >= 0.1 TMPCM: FM <= 0.9 TMPCM (:3455)")
    site("CH = KARMAN**2 / (CMFM*CHFH)", c(0.16), cmfm * cmfm, ":3500")
    assert cm_q.lo >= cm.lo * (1 - 1e-4) and cm_q.hi <= cm.hi * (1 + 1e-4)
    sqrt_site("FV = UR*SQRT(CM)", cm, ":3502", "also bare_flux's sfcdif1")
    # ---- vege_flux: canopy resistance, :2775 ----
    site("RAHC: 1 / (CH*UR)", c(1.0), cm * ur, ":2775", "then MAX(1, .)")
    # ---- ragrb (iter >= 2), :3301-3306 ----
    gt = site("GRAV / TAH", c(GRAV), tah, ":3313")
    tmp1g = site("TMP1 = KARMAN*(GRAV/TAH)*HG / RHOCP", KARMAN * gt * hg, rhocp, ":3313")
    tmp1g = M(1e-6, tmp1g.hi)
    molg = site("MOLG = -FV**3 / TMP1", fv3, tmp1g, ":3315")
    dzg = diff(zpd.nz(), z0)                        # ZPD - Z0MG, nonzero >= granularity
    dzg = M(dzg.lo, D["HCAN_HI"] + D["Z0_HI"], True)
    mozg = site("MOZG = (ZPD-Z0MG) / MOLG", dzg, molg, ":3316", "then MIN(., 1)")
    fhg_lo = (1.0 + 15.0 * mozg.hi) ** -0.25        # (1 - 15 MOZG)**-0.25, MOZG < 0
    fhg = M(fhg_lo, 5.7)                            # 1 + 4.7 MOZG <= 5.7; averages stay inside
    sqrt_site("CWPC = SQRT(CWP*VAI*HCAN*FHG)", cwph * fhg, ":3343")
    cwpc = fn(math.sqrt, cwph * fhg)                # SQRT(CWP*VAI*HCAN*FHG)
    a14 = cwpc * z0
    q14 = site("CWPC*Z0HG / HCAN", a14, hcan, ":3334", "Z0MG <= HCAN checked: <= CWPC")
    q14 = M(q14.lo, cwpc.hi)
    q15 = site("CWPC*(Z0H+ZPD) / HCAN", cwpc * z0, hcan, ":3335",
               "Z0M + ZPD <= 2 HCAN checked: <= 2 CWPC")
    q15 = M(q15.lo, 2 * cwpc.hi)
    tmp1e = M(math.exp(-q14.hi), 1.0)
    tmp2e = M(math.exp(-q15.hi), 1.0)
    rah2a = site("HCAN*EXP(CWPC) / CWPC", hcan * fn(math.exp, cwpc), cwpc, ":3336")
    # |TMP1 - TMP2|: the sign is not assumed (the kernel does not check
    # Z0MG <= Z0M + ZPD).  Nonzero, the difference is at least the granularity
    # of the smaller exponential; a negative RAHG fails the RAHG window below
    # and the lane re-runs with IEEE division.
    dtmp = M(2.0 ** (math.floor(math.log2(tmp2e.lo)) - 23), 1.0, True)
    kh = M(1e-6, KARMAN * fv.hi * D["HCAN_HI"])    # MAX(KARMAN*FV*(HCAN-ZPD), MPE)
    site("RAHG = TMPRAH2 / KH", rah2a * dtmp, kh, ":3341", "then checked in [RAHG_LO, RAHG_HI]")
    den_rb = M(-math.expm1(-cwpc.lo / 2) * 0.999, -math.expm1(-cwpc.hi / 2))
    site("TMPRB = CWPC*50 / (1-EXP(-CWPC/2))", 50 * cwpc, den_rb, ":3346")
    # 50x / (1 - exp(-x/2)) increases with x, from 100 at x -> 0
    tmprb = M(99.0, 50 * cwpc.hi / -math.expm1(-cwpc.hi / 2) * 1.001)
    rb = tmprb * sdl
    rahg = rahg_w
    # ---- vege_flux body, :2808-2870 ----
    cah = site("CAH = 1 / RAHC", c(1.0), rahc, ":2817")
    cvh = site("CVH = 2*VAIE / RB", 2 * vaie, rb, ":2818")
    cgh = site("CGH = 1 / RAHG", c(1.0), rahg, ":2819")
    cond = cah + cvh + cgh
    site("ATA = (SFCTMP*CAH + TG*CGH) / COND", T * cah + T * cgh, cond, ":2821")
    site("BTA = CVH / COND", cvh, cond, ":2822")
    site("CAW = 1 / RAWC", c(1.0), rahc, ":2826")
    cew = site("CEW = FWET*VAIE / RB", fwet * vaie, rb, ":2827")
    rbrs = M(rb.lo, rb.hi + rs_hi)
    t1 = site("LAISUNE / (RB+RSSUN)", lai, rbrs, ":2828", "RSSUN, RSSHA <= RS_HI checked")
    site("LAISHAE / (RB+RSSHA)", lai, rbrs, ":2828")
    # CTW = (1-FWET)*(...): its bound matters only through BEA's numerator
    # CEW + CTW, which is CTW = the two terms when FWET = 0 and >= CEW otherwise
    ctw = M(t1.lo, 2 * t1.hi, True)
    cgw = site("CGW = 1 / (RAWG+RSURF)", c(1.0), M(rahg.lo, rahg.hi + rsurf_hi), ":2829")
    cond2 = cah + cew + ctw + cgw
    site("AEA = (EAIR*CAW + ESTG*CGW) / COND", M(es.lo * cgw.lo, eair_hi + es.hi * cgw.hi), cond2,
         ":2831")
    bea = site("BEA = (CEW+CTW) / COND", M(min(cew.lo, ctw.lo), cew.hi + ctw.hi, True), cond2,
               ":2832", "FWET = 0: CTW = the LAI terms; FWET > 0: >= CEW")
    one_m_bea = M(2.0 ** -24, 1.0, True)            # BEA <= 1; 1 - BEA is 0 or >= 2^-24
    cev = site("CEV = (1-BEA)*CEW*RHOAIR*CPAIR / GAMMAV", one_m_bea * cew * rhocp, gammav, ":2833")
    # EAH = AEA + BEA*ESTV lies between 0 and max(EAIR, ESTG, ESTV); ESTV >= es.lo, so
    # ESTV - EAH is 0 or >= 2^(E - 23) with E the exponent of es.lo / 2
    de = M(2.0 ** (math.floor(math.log2(es.lo / 2)) - 23), max(es.hi, eair_hi), True)
    site("EVC = FVEG*RHOAIR*CPAIR*CEW*(ESTV-EAH) / GAMMAV", fveg * rhocp * cew * de, gammav,
         ":2842")
    eah = M(es.lo * cgw.lo / cond2.hi, max(es.hi, eair_hi))
    h_q = site("H = RHOAIR*CPAIR*(TAH-SFCTMP) / RAHC", rhocp * dT, rahc, ":2864")
    hg_q = site("HG = RHOAIR*CPAIR*(TG-TAH) / RAHG", rhocp * dT, rahg, ":2865")
    site("QSFC = 0.622*EAH / (SFCPRS-0.378*EAH)", 0.622 * eah,
         M(p.lo - 0.378 * eah.hi, p.hi), ":2868")
    # ---- CTR, TR, DTV = B/A (NMP_VD_CHECKED): the numerators are checked per
    # lane every iteration (vege_domain.h NUM_LO_EXP / NUM_HI_EXP); the
    # denominators are bounded here.  A = FVEG*(4*CIR*TV**3 + CSH + (CEV+CTR)*DESTV),
    # every term >= 0: CIR = (2 - EMV*(1-EMG))*EMV*SB with EMG in [0, 1] (checked)
    # and EMV = 1 - EXP(-VAI), VAI = VAIE*FVEG >= VAI_LO*FVEG_LO; CSH =
    # (1-BTA)*RHOAIR*CPAIR*CVH <= RHOAIR*CPAIR*CVH; CTR <= RHOAIR*CPAIR*CTW / GAMMAV. ----
    numw = M(2.0 ** D["NUM_LO_EXP"] * (1 + 2 * W), 2.0 ** D["NUM_HI_EXP"], True)
    note = "numerator window checked per lane, IEEE loop outside"
    site("CTR = (1-BEA)*CTW*RHOAIR*CPAIR / GAMMAV", numw, gammav, ":2834", note)
    site("TR = FVEG*RHOAIR*CPAIR*CTW*(ESTV-EAH) / GAMMAV", numw, gammav, ":2843", note)
    emv = M(-math.expm1(-D["VAI_LO"] * D["FVEG_LO"]) * 0.9, 1.0)  # fp32 rounding of 1 - EXP(-x) near 1: < 6e-8
    cir = M(emv.lo * SB, 2 * SB)
    ctr_hi = rhocp.hi * ctw.hi / gammav.lo
    a_v = M(fveg.lo * 4 * cir.lo * T.lo ** 3,
            4 * cir.hi * T.hi ** 3 + rhocp.hi * cvh.hi + (cev.hi + ctr_hi) * des.hi)
    site("DTV = B / A", numw, a_v, ":2852", note)
    # ---- bare_flux's Newton loop (:3120-3200; sflx_kernel.hip bare_loop) ----
    # Same sfcdif1 sites with Z0H = Z0MG and ZPD = ZPDG (the snow depth): the
    # kernel checks the same limits on TMPCM.., ZLVL-ZPDG, Z0MG, SFCTMP, air,
    # pressure and wind, and TGB at the start of every iteration.  Its H is
    # CSH*(TGB-SFCTMP) with CSH = RHOAIR*CPAIR/RAHB, RAHB in RAHC's interval, so
    # H has the canopy loop's interval and every sfcdif1 bound above carries over.
    rahb = rahc
    hb = M((rhocp * dT).lo / rahb.hi, (rhocp * dT).hi, True)
    assert hb.lo >= h.lo * 0.999 and hb.hi <= h.hi * 1.001
    site("bare: RAHB: 1 / (CH*UR)", c(1.0), cm * ur, ":3167", "then MAX(1, .)")
    site("bare: EHB = 1 / RAHB", c(1.0), rahb, ":3172")
    site("bare: CSH = RHOAIR*CPAIR / RAHB", rhocp, rahb, ":3186")
    gammag = gammav                                  # same formula with LATHEAG
    cevi = site("bare: RHOAIR*CPAIR / GAMMA", rhocp, gammag, ":3187")
    cevb = site("bare: CEV = (...) / (RSURF+RAWB)", cevi, M(rahb.lo, rahb.hi + rsurf_hi), ":3187")
    # A = 4*CIR*TGB**3 + CSH + CEV*DESTG + CGH, every term >= 0 (CIR = EMG*SB,
    # EMG in [0, 1] and CGH in [0, CGH_HI] checked per column): >= CSH
    a_b = M(rhocp.lo / rahb.hi,
            4 * SB * T.hi ** 3 + rhocp.hi / rahb.lo + cevb.hi * des.hi + D["CGH_HI"])
    site("bare: DTG = B / A", numw, a_b, ":3198", note)

    stomata_sites(D, T, p, es, rb)
    soil_sites()

    # ---- induction: the iteration ends inside the intervals it started from ----
    assert h_q.hi <= h.hi * 1.001 and h_q.lo >= h.lo * 0.999, (h_q, h)
    assert hg_q.hi <= hg.hi * 1.001 and hg_q.lo >= hg.lo * 0.999, (hg_q, hg)
    assert eah.hi <= max(es.hi, eair_hi) * 1.001
    assert p.lo - 0.378 * eah.hi > 0

    print(f"domain: {HDR}")
    print(f"exact region: |b| in [2^-126, 2^126], a = 0 or |a| >= 2^-102, |a/b| in [2^-126, 2^126]; "
          f"sqrt: x finite and >= 2^-96")
    print(f"{'site':46s} {'func.f90':8s} {'|a|':>22s} {'|b|':>22s} {'|a/b|':>22s}  ok")
    for name, ref, a, b, q, ok, note in rows:
        print(f"{name:46s} {ref:8s} {a!r:>22s} {b!r:>22s} {q!r:>22s}  {'yes' if ok else 'NO'}"
              + (f"  ({note})" if note else ""))
    print(f"derived: FHG >= {fhg_lo:.3g}, CWPC in {cwpc!r}, FV in {fv!r}, RAHC in {rahc!r}, "
          f"RB in {rb!r}")
    if bad:
        print("FAILED:", bad)
        return 1
    print(f"all {len(rows)} sites inside the exact region")
    return 0


if __name__ == "__main__":
    sys.exit(main())
