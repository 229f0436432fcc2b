/*
 * ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
 *
 * Plain-C restatement of the reference noahmp_sflx time step
 * (/root/reference/core/module_noahmp_func.f90).  Every function cites the
 * reference lines it follows.  The arithmetic keeps the reference's
 * evaluation order, single-precision literals and the exponent lowering flang
 * applies (x**n and x**2.0/x**3.0 -> repeated products, x**0.5 -> sqrt,
 * 2.0**x -> exp2, other real exponents -> pow), so the fp32 build can follow
 * the fp32 reference bit for bit on glibc.
 *
 * Array conventions: snow/soil arrays (-2:4) are pointers into a 7-element
 * buffer at offset 2 (X[-2..4]); soil-only arrays (1:4) are 5-element
 * buffers used 1-based; snow-only arrays (-2:0) are pointers at offset 2.
 */
#include "noahmp_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef ORACLE_REAL real;

#define ORACLE_IS_FLOAT (sizeof(real) == 4)
#define K(x) ((real)(ORACLE_IS_FLOAT ? (double)(x##f) : (x)))

/* Loop trip counts per column (tools/iter_stats.py; build with -DORACLE_ITER_STATS
 * only): 0 vege_flux Newton, 1 stomata bisection, 2 frh2o, 3 soilwater
 * sub-steps, 4 bare_flux Newton. */
#ifdef ORACLE_ITER_STATS
static int32_t* g_stats;
static int32_t g_stat_col;
void oracle_set_stats(int32_t* buf) { g_stats = buf; }
#define ITER_STAT(k)                                        \
  do {                                                      \
    if (g_stats) g_stats[(size_t)g_stat_col * 8 + (k)]++;   \
  } while (0)
#else
#define ITER_STAT(k) ((void)0)
#endif

/* Division operand ranges of the canopy Newton loop (vege_flux with sfcdif1
 * and ragrb; build with -DORACLE_DIV_STATS only, tools/div_ranges.py): per
 * site the smallest / largest |a|, |b|, |a/b| over nonzero finite values and
 * the count of zero numerators.  The arithmetic is unchanged: DV(k, a, b) is
 * a / b. */
#ifdef ORACLE_DIV_STATS
#define NDIVSITE 40
static double g_div[NDIVSITE][8];
static int g_div_init;
void oracle_div_stats(double* out, int reset) {
  if (!g_div_init || reset) {
    for (int k = 0; k < NDIVSITE; ++k) {
      g_div[k][0] = g_div[k][2] = g_div[k][4] = INFINITY;
      g_div[k][1] = g_div[k][3] = g_div[k][5] = 0.0;
      g_div[k][6] = g_div[k][7] = 0.0;
    }
    g_div_init = 1;
  }
  if (out) memcpy(out, g_div, sizeof(g_div));
}
static inline void div_rec(int k, double v, int slot) {
  v = fabs(v);
  if (v == 0.0 || !isfinite(v)) return;
  if (v < g_div[k][slot]) g_div[k][slot] = v;
  if (v > g_div[k][slot + 1]) g_div[k][slot + 1] = v;
}
static inline real div_stat(int k, real a, real b) {
  if (!g_div_init) oracle_div_stats(NULL, 1);
  const real q = a / b;
  div_rec(k, a, 0);
  div_rec(k, b, 2);
  div_rec(k, q, 4);
  g_div[k][6] += 1.0;
  if (a == 0) g_div[k][7] += 1.0;
  return q;
}
#define DV(k, a, b) div_stat((k), (a), (b))
#else
#define DV(k, a, b) ((a) / (b))
#endif

#if defined(ORACLE_DOUBLE)
#define EXP exp
#define LOG log
#define LOG10 log10
#define POW pow
#define SQRT sqrt
#define TANH tanh
#define ATAN atan
#define TAN tan
#define ACOS acos
#define COS cos
#define FABS fabs
#define FMOD fmod
#define EXP2 exp2
#define COPYSIGN copysign
#elif defined(ORACLE_CRMATH)
/* fp32 arithmetic with correctly rounded elementary functions (evaluated in
 * double, rounded once) instead of glibc's float libm.  Isolates libm
 * rounding from the algorithm: the GPU engine's default math mode computes
 * exactly this, so GPU-vs-CR differences mean a kernel bug, while CR-vs-
 * reference differences are glibc float-libm ulps (tanhf/atanf chiefly). */
static inline float cr_exp(float x) { return (float)exp((double)x); }
static inline float cr_log(float x) { return (float)log((double)x); }
static inline float cr_log10(float x) { return (float)log10((double)x); }
static inline float cr_pow(float x, float y) { return (float)pow((double)x, (double)y); }
static inline float cr_tanh(float x) { return (float)tanh((double)x); }
static inline float cr_atan(float x) { return (float)atan((double)x); }
static inline float cr_tan(float x) { return (float)tan((double)x); }
static inline float cr_acos(float x) { return (float)acos((double)x); }
static inline float cr_cos(float x) { return (float)cos((double)x); }
static inline float cr_exp2(float x) { return (float)exp2((double)x); }
#define EXP cr_exp
#define LOG cr_log
#define LOG10 cr_log10
#define POW cr_pow
#define SQRT sqrtf
#define TANH cr_tanh
#define ATAN cr_atan
#define TAN cr_tan
#define ACOS cr_acos
#define COS cr_cos
#define FABS fabsf
#define FMOD fmodf
#define EXP2 cr_exp2
#define COPYSIGN copysignf
#else
#define EXP expf
#define LOG logf
#define LOG10 log10f
#define POW powf
#define SQRT sqrtf
#define TANH tanhf
#define ATAN atanf
#define TAN tanf
#define ACOS acosf
#define COS cosf
#define FABS fabsf
#define FMOD fmodf
#define EXP2 exp2f
#define COPYSIGN copysignf
#endif

#define NSOIL 4
#define NSNOW 3

static inline real rmax(real a, real b) { return a > b ? a : b; }
static inline real rmin(real a, real b) { return a < b ? a : b; }
static inline real p2(real x) { return x * x; }
static inline real p3(real x) { return x * (x * x); }
static inline real p4(real x) { return x * p3(x); }
static inline real p5(real x) { return x * p4(x); }

/* ---- constants: core/module_noahmp_const.f90:14-35 ---- */
#define MPE K(1.0E-6)
#define GRAV K(9.80616)
#define SB K(5.67E-8)
#define RGAS K(8.3144598)
#define KARMAN K(0.40)
#define TFRZ K(273.15)
#define HSUB K(2.8440E6)
#define HVAP K(2.5104E6)
#define HFUS K(0.3336E6)
#define CWAT K(4.188E6)
#define CICE K(2.094E6)
#define CPAIR K(1004.64)
#define TKWAT K(0.6)
#define TKICE K(2.2)
#define RAIR K(287.04)
#define RVAP K(461.269)
#define DENWAT K(1000.0)
#define DENICE K(917.0)

/* table accessors (1-based type indices as in the reference) */
#define SOILP(f) ((real)P->f[sltyp - 1])
#define VEGP(f) ((real)P->f[lutyp - 1])

typedef struct {
  const nmp_params* P;
  const nmp_options* O;
  int32_t status;
} ctx_t;

/* ------------------------------------------------------------------------ */
/* atm: func.f90:479-531 */
static void atm(real SFCPRS, real SFCTMP, real Q2, real PRCP, real SOLDN, real COSZ,
                real* THAIR, real* QAIR, real* EAIR, real* RHOAIR, real* QPRECC, real* QPRECL,
                real SOLAD[2], real SOLAI[2], real* SWDOWN) {
  real PAIR = SFCPRS;
  *THAIR = SFCTMP * POW(SFCPRS / PAIR, RAIR / CPAIR);
  *QAIR = Q2;
  *EAIR = *QAIR * SFCPRS / (K(0.622) + K(0.378) * *QAIR);
  *RHOAIR = (SFCPRS - K(0.378) * *EAIR) / (RAIR * SFCTMP);
  *QPRECC = K(0.10) * PRCP;
  *QPRECL = K(0.90) * PRCP;
  *SWDOWN = (COSZ <= K(0.0)) ? K(0.0) : SOLDN;
  SOLAD[0] = *SWDOWN * K(0.7) * K(0.5);
  SOLAD[1] = *SWDOWN * K(0.7) * K(0.5);
  SOLAI[0] = *SWDOWN * K(0.3) * K(0.5);
  SOLAI[1] = *SWDOWN * K(0.3) * K(0.5);
}

/* phenology: func.f90:534-630 */
static void phenology(ctx_t* X, int lutyp, real snowh, real TV, real LAT, int YEARLEN,
                      real JULIAN, real* LAI, real* SAI, real* HTOP, real* elai, real* esai,
                      real* IGS) {
  const nmp_params* P = X->P;
  int ov = X->O->opt_veg;
  if (ov == 1 || ov == 3 || ov == 4) {
    real DAY = (LAT >= K(0.0)) ? JULIAN
                               : FMOD(JULIAN + (K(0.5) * (real)YEARLEN), (real)YEARLEN);
    real T = K(12.0) * DAY / (real)YEARLEN;
    int IT1 = (int)(T + K(0.5));
    int IT2 = IT1 + 1;
    real WT1 = ((real)IT1 + K(0.5)) - T;
    real WT2 = K(1.0) - WT1;
    if (IT1 < 1) IT1 = 12;
    if (IT2 > 12) IT2 = 1;
    *LAI = WT1 * (real)P->lai12m[lutyp - 1][IT1 - 1] + WT2 * (real)P->lai12m[lutyp - 1][IT2 - 1];
    *SAI = WT1 * (real)P->sai12m[lutyp - 1][IT1 - 1] + WT2 * (real)P->sai12m[lutyp - 1][IT2 - 1];
  }
  if (*SAI < K(0.05)) *SAI = K(0.0);
  if (*LAI < K(0.05) || *SAI == K(0.0)) *LAI = K(0.0);
  if (lutyp == P->iswater || lutyp == P->isbarren || lutyp == P->isice || lutyp == P->isurban) {
    *LAI = K(0.0);
    *SAI = K(0.0);
  }
  real HVT = VEGP(hvt), HVB = VEGP(hvb);
  real DB = rmin(rmax(snowh - HVB, K(0.0)), HVT - HVB);
  real FB = DB / rmax(K(1.0E-06), HVT - HVB);
  if (HVT > K(0.0) && HVT <= K(1.0)) {
    real snowhc = HVT * EXP(-snowh / K(0.2));
    FB = rmin(snowh, snowhc) / snowhc;
  }
  *elai = *LAI * (K(1.0) - FB);
  *esai = *SAI * (K(1.0) - FB);
  if (*esai < K(0.05)) *esai = K(0.0);
  if (*elai < K(0.05) || *esai == K(0.0)) *elai = K(0.0);
  *IGS = (TV > VEGP(tmin)) ? K(1.0) : K(0.0);
  *HTOP = HVT;
}

/* esat: func.f90:3692-3736 */
static void esat(real T, real* ESW, real* ESI, real* DESW, real* DESI) {
  const real A0 = K(6.107799961), A1 = K(4.436518521E-01), A2 = K(1.428945805E-02),
             A3 = K(2.650648471E-04), A4 = K(3.031240396E-06), A5 = K(2.034080948E-08),
             A6 = K(6.136820929E-11);
  const real B0 = K(6.109177956), B1 = K(5.034698970E-01), B2 = K(1.886013408E-02),
             B3 = K(4.176223716E-04), B4 = K(5.824720280E-06), B5 = K(4.838803174E-08),
             B6 = K(1.838826904E-10);
  const real C0 = K(4.438099984E-01), C1 = K(2.857002636E-02), C2 = K(7.938054040E-04),
             C3 = K(1.215215065E-05), C4 = K(1.036561403E-07), C5 = K(3.532421810e-10),
             C6 = K(-7.090244804E-13);
  const real D0 = K(5.030305237E-01), D1 = K(3.773255020E-02), D2 = K(1.267995369E-03),
             D3 = K(2.477563108E-05), D4 = K(3.005693132E-07), D5 = K(2.158542548E-09),
             D6 = K(7.131097725E-12);
  *ESW = K(100.) * (A0 + T * (A1 + T * (A2 + T * (A3 + T * (A4 + T * (A5 + T * A6))))));
  *ESI = K(100.) * (B0 + T * (B1 + T * (B2 + T * (B3 + T * (B4 + T * (B5 + T * B6))))));
  *DESW = K(100.) * (C0 + T * (C1 + T * (C2 + T * (C3 + T * (C4 + T * (C5 + T * C6))))));
  *DESI = K(100.) * (D0 + T * (D1 + T * (D2 + T * (D3 + T * (D4 + T * (D5 + T * D6))))));
}

static inline real tdc(real T) { return rmin(K(50.0), rmax(K(-50.0), (T - TFRZ))); }

/* csnow: func.f90:1448-1497 */
static void csnow(int ISNOW, const real* SNICE, const real* SNLIQ, const real* DZSNSO,
                  real* TKSNO, real* CVSNO, real* SNICEV, real* SNLIQV, real* epore) {
  real BDSNOIb[3];
  real* BDSNOI = BDSNOIb + 2;
  for (int IZ = ISNOW + 1; IZ <= 0; ++IZ) {
    SNICEV[IZ] = rmin(K(1.0), SNICE[IZ] / (DZSNSO[IZ] * DENICE));
    epore[IZ] = K(1.0) - SNICEV[IZ];
    SNLIQV[IZ] = rmin(epore[IZ], SNLIQ[IZ] / (DZSNSO[IZ] * DENWAT));
  }
  for (int IZ = ISNOW + 1; IZ <= 0; ++IZ) {
    BDSNOI[IZ] = (SNICE[IZ] + SNLIQ[IZ]) / DZSNSO[IZ];
    CVSNO[IZ] = CICE * SNICEV[IZ] + CWAT * SNLIQV[IZ];
  }
  for (int IZ = ISNOW + 1; IZ <= 0; ++IZ) TKSNO[IZ] = K(3.2217E-6) * p2(BDSNOI[IZ]);
}

/* tdfcnd: func.f90:1500-1595 */
static real tdfcnd(const nmp_params* P, int sltyp, real SMC, real soilwat) {
  real SATRATIO = SMC / SOILP(smcmax);
  real THKW = K(0.57);
  real THKQTZ = K(7.7);
  /* THKO = 2.0: pow(2.0, x) is lowered to exp2 by the reference's compiler */
  real THKS = POW(THKQTZ, SOILP(quartz)) * EXP2(K(1.0) - SOILP(quartz));
  real XUNFROZ = soilwat / SMC;
  real XU = XUNFROZ * SOILP(smcmax);
  real THKSAT = POW(THKS, K(1.0) - SOILP(smcmax)) * POW(TKICE, SOILP(smcmax) - XU) * POW(THKW, XU);
  real GAMMD = (K(1.0) - SOILP(smcmax)) * K(2700.0);
  real THKDRY = (K(0.135) * GAMMD + K(64.7)) / (K(2700.0) - K(0.947) * GAMMD);
  real AKE;
  if ((soilwat + K(0.0005)) < SMC) {
    AKE = SATRATIO;
  } else {
    AKE = (SATRATIO > K(0.1)) ? LOG10(SATRATIO) + K(1.0) : K(0.0);
  }
  return AKE * (THKSAT - THKDRY) + THKDRY;
}

/* thermoprop: func.f90:1341-1445 */
static void thermoprop(ctx_t* X, int sltyp, int lutyp, int ISNOW, int IST, const real* DZSNSO,
                       real DT, real snowh, const real* SNICE, const real* SNLIQ, real CSOIL,
                       const real* SMC, const real* soilwat, const real* STC, real* DF,
                       real* HCPCT, real* SNICEV, real* SNLIQV, real* epore, real* FACT) {
  const nmp_params* P = X->P;
  real CVSNOb[3], TKSNOb[3];
  real *CVSNO = CVSNOb + 2, *TKSNO = TKSNOb + 2;
  csnow(ISNOW, SNICE, SNLIQ, DZSNSO, TKSNO, CVSNO, SNICEV, SNLIQV, epore);
  for (int IZ = ISNOW + 1; IZ <= 0; ++IZ) {
    DF[IZ] = TKSNO[IZ];
    HCPCT[IZ] = CVSNO[IZ];
  }
  for (int IZ = 1; IZ <= NSOIL; ++IZ) {
    real soilice = SMC[IZ] - soilwat[IZ];
    HCPCT[IZ] = soilwat[IZ] * CWAT + (K(1.0) - SOILP(smcmax)) * CSOIL +
                (SOILP(smcmax) - SMC[IZ]) * CPAIR + soilice * CICE;
    DF[IZ] = tdfcnd(P, sltyp, SMC[IZ], soilwat[IZ]);
  }
  if (lutyp == P->isurban)
    for (int IZ = 1; IZ <= NSOIL; ++IZ) DF[IZ] = K(3.24);
  if (IST == 2) {
    for (int IZ = 1; IZ <= NSOIL; ++IZ) {
      if (STC[IZ] > TFRZ) {
        HCPCT[IZ] = CWAT;
        DF[IZ] = TKWAT;
      } else {
        HCPCT[IZ] = CICE;
        DF[IZ] = TKICE;
      }
    }
  }
  for (int IZ = ISNOW + 1; IZ <= NSOIL; ++IZ) FACT[IZ] = DT / (HCPCT[IZ] * DZSNSO[IZ]);
  if (ISNOW == 0)
    DF[1] = (DF[1] * DZSNSO[1] + K(0.35) * snowh) / (snowh + DZSNSO[1]);
  else
    DF[1] = (DF[1] * DZSNSO[1] + DF[0] * DZSNSO[0]) / (DZSNSO[0] + DZSNSO[1]);
}

/* snowage: func.f90:2008-2054 */
static void snowage(const nmp_params* P, real DT, real TG, real SNEQVO, real sneqv, real* TAUSS,
                    real* FAGE) {
  if (sneqv <= K(0.0)) {
    *TAUSS = K(0.0);
  } else if (sneqv > K(800.0)) {
    *TAUSS = K(0.0);
  } else {
    real DELA0 = K(1.0E-6) * DT;
    real ARG = K(5.0E3) * (K(1.0) / TFRZ - K(1.0) / TG);
    real AGE1 = EXP(ARG);
    real AGE2 = EXP(rmin(K(0.0), K(10.0) * ARG));
    real AGE3 = K(0.3);
    real TAGE = AGE1 + AGE2 + AGE3;
    real DELA = DELA0 * TAGE;
    real DELS = rmax(K(0.0), sneqv - SNEQVO) / (real)P->swemax;
    real SGE = (*TAUSS + DELA) * (K(1.0) - DELS);
    *TAUSS = rmax(K(0.0), SGE);
  }
  *FAGE = *TAUSS / (*TAUSS + K(1.0));
}

/* snowalb_bats: func.f90:2057-2102 */
static void snowalb_bats(real COSZ, real FAGE, real ALBSND[2], real ALBSNI[2]) {
  const real C1 = K(0.2), C2 = K(0.5);
  real SL = K(2.0);
  real SL1 = K(1.0) / SL;
  real SL2 = K(2.0) * SL;
  real CF1 = ((K(1.0) + SL1) / (K(1.0) + SL2 * COSZ) - SL1);
  real FZEN = rmax(CF1, K(0.0));
  ALBSNI[0] = K(0.95) * (K(1.0) - C1 * FAGE);
  ALBSNI[1] = K(0.65) * (K(1.0) - C2 * FAGE);
  ALBSND[0] = ALBSNI[0] + K(0.4) * FZEN * (K(1.0) - ALBSNI[0]);
  ALBSND[1] = ALBSNI[1] + K(0.4) * FZEN * (K(1.0) - ALBSNI[1]);
}

/* snowalb_class: func.f90:2105-2151 */
static real snowalb_class(const nmp_params* P, real QSNOW, real DT, real ALBOLD, real ALBSND[2],
                          real ALBSNI[2]) {
  real ALB = K(0.55) + (ALBOLD - K(0.55)) * EXP(-K(0.01) * DT / K(3600.0));
  if (QSNOW > K(0.0))
    ALB = ALB + rmin(QSNOW * DT, (real)P->swemax) * (K(0.84) - ALB) / (real)P->swemax;
  ALBSNI[0] = ALB;
  ALBSNI[1] = ALB;
  ALBSND[0] = ALB;
  ALBSND[1] = ALB;
  return ALB;
}

/* groundalb: func.f90:2154-2212 */
static void groundalb(const nmp_params* P, int IST, int ISC, real FSNO, const real* SMC,
                      const real ALBSND[2], const real ALBSNI[2], real COSZ, real TG,
                      real ALBGRD[2], real ALBGRI[2]) {
  for (int IB = 0; IB < 2; ++IB) {
    real INC = rmax(K(0.11) - K(0.40) * SMC[1], K(0.0));
    real ALBSOD, ALBSOI;
    if (IST == 1) {
      ALBSOD = rmin((real)P->albsat[ISC - 1][IB] + INC, (real)P->albdry[ISC - 1][IB]);
      ALBSOI = ALBSOD;
    } else if (TG > TFRZ) {
      ALBSOD = K(0.06) / (POW(rmax(K(0.01), COSZ), K(1.7)) + K(0.15));
      ALBSOI = K(0.06);
    } else {
      ALBSOD = (real)P->alblake[IB];
      ALBSOI = ALBSOD;
    }
    if (IST == 1 && ISC == 9) {
      ALBSOD = ALBSOD + K(0.10);
      ALBSOI = ALBSOI + K(0.10);
    }
    ALBGRD[IB] = ALBSOD * (K(1.0) - FSNO) + ALBSND[IB] * FSNO;
    ALBGRI[IB] = ALBSOI * (K(1.0) - FSNO) + ALBSNI[IB] * FSNO;
  }
}

/* twostream: func.f90:2215-2462 (one band IB, one beam type IC) */
static void twostream(ctx_t* X, int lutyp, int IB, int IC, real COSZ, real VAI, real FWET, real T,
                      const real ALBGRD[2], const real ALBGRI[2], const real RHO[2],
                      const real TAU[2], real fveg, real* FAB, real* FRE, real* FTD, real* FTI,
                      real* GDIR, real* FREV, real* FREG, real* BGAP, real* WGAP) {
  const nmp_params* P = X->P;
  const real PAI = K(3.14159265);
  real GAP = K(0.0), KOPEN = K(0.0);
  if (VAI == K(0.0)) {
    GAP = K(1.0);
    KOPEN = K(1.0);
  } else {
    int orad = X->O->opt_rad;
    if (orad == 1) {
      real RC = VEGP(rcrown);
      real DENfveg = -LOG(rmax(K(1.0) - fveg, K(0.01))) / (PAI * p2(RC));
      real HD = VEGP(hvt) - VEGP(hvb);
      real BB = K(0.5) * HD;
      real THETAP = ATAN(BB / RC * TAN(ACOS(rmax(K(0.01), COSZ))));
      *BGAP = EXP(-DENfveg * PAI * p2(RC) / COS(THETAP));
      real FA = VAI / (K(1.33) * PAI * p3(RC) * (BB / RC) * DENfveg);
      real NEWVAI = HD * FA;
      *WGAP = (K(1.0) - *BGAP) * EXP(-K(0.5) * NEWVAI / COSZ);
      GAP = rmin(K(1.0) - fveg, *BGAP + *WGAP);
      KOPEN = K(0.05);
    }
    if (orad == 2) {
      GAP = K(0.0);
      KOPEN = K(0.0);
    }
    if (orad == 3) {
      GAP = K(1.0) - fveg;
      KOPEN = K(1.0) - fveg;
    }
  }
  real COSZI = rmax(K(0.001), COSZ);
  real CHIL = rmin(rmax(VEGP(xl), K(-0.4)), K(0.6));
  if (FABS(CHIL) <= K(0.01)) CHIL = K(0.01);
  real PHI1 = K(0.5) - K(0.633) * CHIL - K(0.330) * CHIL * CHIL;
  real PHI2 = K(0.877) * (K(1.) - K(2.) * PHI1);
  *GDIR = PHI1 + PHI2 * COSZI;
  real EXT = *GDIR / COSZI;
  real AVMU = (K(1.) - PHI1 / PHI2 * LOG((PHI1 + PHI2) / PHI1)) / PHI2;
  real OMEGAL = RHO[IB] + TAU[IB];
  real TMP0 = *GDIR + PHI2 * COSZI;
  real TMP1 = PHI1 * COSZI;
  real ASU = K(0.5) * OMEGAL * *GDIR / TMP0 * (K(1.) - TMP1 / TMP0 * LOG((TMP1 + TMP0) / TMP1));
  real BETADL = (K(1.) + AVMU * EXT) / (OMEGAL * AVMU * EXT) * ASU;
  real BETAIL = K(0.5) * (RHO[IB] + TAU[IB] + (RHO[IB] - TAU[IB]) * p2((K(1.) + CHIL) / K(2.))) /
                OMEGAL;
  real TMP2;
  if (T > TFRZ) {
    TMP0 = OMEGAL;
    TMP1 = BETADL;
    TMP2 = BETAIL;
  } else {
    real OMS = (real)P->omegas[IB];
    TMP0 = (K(1.0) - FWET) * OMEGAL + FWET * OMS;
    TMP1 = ((K(1.0) - FWET) * OMEGAL * BETADL + FWET * OMS * (real)P->betads) / TMP0;
    TMP2 = ((K(1.0) - FWET) * OMEGAL * BETAIL + FWET * OMS * (real)P->betais) / TMP0;
  }
  real OMEGA = TMP0, BETAD = TMP1, BETAI = TMP2;
  real B = K(1.) - OMEGA + OMEGA * BETAI;
  real C = OMEGA * BETAI;
  TMP0 = AVMU * EXT;
  real D = TMP0 * OMEGA * BETAD;
  real F = TMP0 * OMEGA * (K(1.) - BETAD);
  TMP1 = B * B - C * C;
  real H = SQRT(TMP1) / AVMU;
  real SIGMA = TMP0 * TMP0 - TMP1;
  if (FABS(SIGMA) < K(1.e-6)) SIGMA = COPYSIGN(K(1.e-6), SIGMA);
  real P1 = B + AVMU * H;
  real P2 = B - AVMU * H;
  real P3 = B + TMP0;
  real P4 = B - TMP0;
  real S1 = EXP(-H * VAI);
  real S2 = EXP(-EXT * VAI);
  real U1, U2, U3;
  if (IC == 0) {
    U1 = B - C / ALBGRD[IB];
    U2 = B - C * ALBGRD[IB];
    U3 = F + C * ALBGRD[IB];
  } else {
    U1 = B - C / ALBGRI[IB];
    U2 = B - C * ALBGRI[IB];
    U3 = F + C * ALBGRI[IB];
  }
  TMP2 = U1 - AVMU * H;
  real TMP3 = U1 + AVMU * H;
  real D1 = P1 * TMP2 / S1 - P2 * TMP3 * S1;
  real TMP4 = U2 + AVMU * H;
  real TMP5 = U2 - AVMU * H;
  real D2 = TMP4 / S1 - TMP5 * S1;
  real H1 = -D * P4 - C * F;
  real TMP6 = D - H1 * P3 / SIGMA;
  real TMP7 = (D - C - H1 / SIGMA * (U1 + TMP0)) * S2;
  real H2 = (TMP6 * TMP2 / S1 - P2 * TMP7) / D1;
  real H3 = -(TMP6 * TMP3 * S1 - P1 * TMP7) / D1;
  real H4 = -F * P3 - C * D;
  real TMP8 = H4 / SIGMA;
  real TMP9 = (U3 - TMP8 * (U2 - TMP0)) * S2;
  real H5 = -(TMP8 * TMP4 / S1 + TMP9) / D2;
  real H6 = (TMP8 * TMP5 * S1 + TMP9) / D2;
  real H7 = (C * TMP2) / (D1 * S1);
  real H8 = (-C * TMP3 * S1) / D1;
  real H9 = TMP4 / (D2 * S1);
  real H10 = (-TMP5 * S1) / D2;
  real FTDS, FTIS, FRES, FREVEG, FREBAR;
  if (IC == 0) {
    FTDS = S2 * (K(1.0) - GAP) + GAP;
    FTIS = (H4 * S2 / SIGMA + H5 * S1 + H6 / S1) * (K(1.0) - GAP);
  } else {
    FTDS = K(0.);
    FTIS = (H9 * S1 + H10 / S1) * (K(1.0) - KOPEN) + KOPEN;
  }
  FTD[IB] = FTDS;
  FTI[IB] = FTIS;
  if (IC == 0) {
    FRES = (H1 / SIGMA + H2 + H3) * (K(1.0) - GAP) + ALBGRD[IB] * GAP;
    FREVEG = (H1 / SIGMA + H2 + H3) * (K(1.0) - GAP);
    FREBAR = ALBGRD[IB] * GAP;
  } else {
    FRES = (H7 + H8) * (K(1.0) - KOPEN) + ALBGRI[IB] * KOPEN;
    FREVEG = (H7 + H8) * (K(1.0) - KOPEN) + ALBGRI[IB] * KOPEN;
    FREBAR = K(0.0);
  }
  FRE[IB] = FRES;
  FREV[IB] = FREVEG;
  FREG[IB] = FREBAR;
  FAB[IB] = K(1.0) - FRE[IB] - (K(1.0) - ALBGRD[IB]) * FTD[IB] - (K(1.0) - ALBGRI[IB]) * FTI[IB];
}

/* albedo: func.f90:1717-1887 */
static void albedo(ctx_t* X, int lutyp, int IST, int ISC, real DT, real COSZ, real elai,
                   real esai, real TG, real TV, real FSNO, real FWET, const real* SMC,
                   real SNEQVO, real sneqv, real QSNOW, real fveg, real* ALBOLD, real* TAUSS,
                   real ALBGRD[2], real ALBGRI[2], real ALBD[2], real ALBI[2], real FABD[2],
                   real FABI[2], real FTDD[2], real FTID[2], real FTII[2], real* FSUN,
                   real* BGAP, real* WGAP) {
  const nmp_params* P = X->P;
  real MPEl = K(1.0E-06);
  *BGAP = K(0.0);
  *WGAP = K(0.0);
  for (int IB = 0; IB < 2; ++IB) {
    ALBD[IB] = ALBI[IB] = ALBGRD[IB] = ALBGRI[IB] = K(0.0);
    FABD[IB] = FABI[IB] = FTDD[IB] = FTID[IB] = FTII[IB] = K(0.0);
  }
  *FSUN = K(0.0);
  if (COSZ <= K(0.0)) return;
  real RHO[2], TAU[2], VAI = K(0.0), WL, WS;
  for (int IB = 0; IB < 2; ++IB) {
    VAI = elai + esai;
    WL = elai / rmax(VAI, MPEl);
    WS = esai / rmax(VAI, MPEl);
    RHO[IB] = rmax((real)P->rhol[lutyp - 1][IB] * WL + (real)P->rhos[lutyp - 1][IB] * WS, MPEl);
    TAU[IB] = rmax((real)P->taul[lutyp - 1][IB] * WL + (real)P->taus[lutyp - 1][IB] * WS, MPEl);
  }
  real FAGE;
  snowage(P, DT, TG, SNEQVO, sneqv, TAUSS, &FAGE);
  real ALBSND[2] = {K(0.0), K(0.0)}, ALBSNI[2] = {K(0.0), K(0.0)};
  if (X->O->opt_alb == 1) snowalb_bats(COSZ, FAGE, ALBSND, ALBSNI);
  if (X->O->opt_alb == 2) *ALBOLD = snowalb_class(P, QSNOW, DT, *ALBOLD, ALBSND, ALBSNI);
  groundalb(P, IST, ISC, FSNO, SMC, ALBSND, ALBSNI, COSZ, TG, ALBGRD, ALBGRI);
  real GDIR = K(0.0), FTDI[2], FREVD[2], FREGD[2], FREVI[2], FREGI[2];
  for (int IB = 0; IB < 2; ++IB) {
    twostream(X, lutyp, IB, 0, COSZ, VAI, FWET, TV, ALBGRD, ALBGRI, RHO, TAU, fveg, FABD, ALBD,
              FTDD, FTID, &GDIR, FREVD, FREGD, BGAP, WGAP);
    twostream(X, lutyp, IB, 1, COSZ, VAI, FWET, TV, ALBGRD, ALBGRI, RHO, TAU, fveg, FABI, ALBI,
              FTDI, FTII, &GDIR, FREVI, FREGI, BGAP, WGAP);
  }
  real EXT = GDIR / COSZ * SQRT(K(1.0) - RHO[0] - TAU[0]);
  *FSUN = (K(1.0) - EXP(-EXT * VAI)) / rmax(EXT * VAI, MPEl);
  EXT = *FSUN;
  WL = (EXT < K(0.01)) ? K(0.) : EXT;
  *FSUN = WL;
}

/* surrad: func.f90:1890-2005 (FSRV/FSRG omitted: undefined at night, printout only) */
static void surrad(real MPEl, real FSUN, real FSHA, real elai, real VAI, real LAISUN,
                   real LAISHA, const real SOLAD[2], const real SOLAI[2], const real FABD[2],
                   const real FABI[2], const real FTDD[2], const real FTID[2], const real FTII[2],
                   const real ALBGRD[2], const real ALBGRI[2], const real ALBD[2],
                   const real ALBI[2], real* PARSUN, real* PARSHA, real* SAV, real* SAG,
                   real* FSA, real* FSR) {
  real CAD[2], CAI[2];
  *SAG = K(0.0);
  *SAV = K(0.0);
  *FSA = K(0.0);
  for (int IB = 0; IB < 2; ++IB) {
    CAD[IB] = SOLAD[IB] * FABD[IB];
    CAI[IB] = SOLAI[IB] * FABI[IB];
    *SAV = *SAV + CAD[IB] + CAI[IB];
    *FSA = *FSA + CAD[IB] + CAI[IB];
    real TRD = SOLAD[IB] * FTDD[IB];
    real TRI = SOLAD[IB] * FTID[IB] + SOLAI[IB] * FTII[IB];
    real ABS_ = TRD * (K(1.0) - ALBGRD[IB]) + TRI * (K(1.0) - ALBGRI[IB]);
    *SAG = *SAG + ABS_;
    *FSA = *FSA + ABS_;
  }
  real LAIFRA = elai / rmax(VAI, MPEl);
  if (FSUN > K(0.0)) {
    *PARSUN = (CAD[0] + FSUN * CAI[0]) * LAIFRA / rmax(LAISUN, MPEl);
    *PARSHA = (FSHA * CAI[0]) * LAIFRA / rmax(LAISHA, MPEl);
  } else {
    *PARSUN = K(0.0);
    *PARSHA = (CAD[0] + CAI[0]) * LAIFRA / rmax(LAISHA, MPEl);
  }
  real RVIS = ALBD[0] * SOLAD[0] + ALBI[0] * SOLAI[0];
  real RNIR = ALBD[1] * SOLAD[1] + ALBI[1] * SOLAI[1];
  *FSR = RVIS + RNIR;
}

/* sfcdif1: func.f90:3353-3508 */
static void sfcdif1(ctx_t* X, int iter, real SFCTMP, real RHOAIR, real H, real QAIR, real ZLVL,
                    real ZPD, real Z0M, real Z0H, real UR, real MPEl, real* MOZ, int* MOZSGN,
                    real* FM, real* FH, real* FM2, real* FH2, real* CM, real* CH, real* FV,
                    real* CH2) {
  real MOZOLD = *MOZ;
  if (ZLVL <= ZPD) X->status |= NMP_ST_ZLVL;
  real TMPCM = LOG((ZLVL - ZPD) / Z0M);
  real TMPCH = LOG((ZLVL - ZPD) / Z0H);
  real TMPCM2 = LOG((K(2.0) + Z0M) / Z0M);
  real TMPCH2 = LOG((K(2.0) + Z0H) / Z0H);
  real MOL, MOZ2;
  if (iter == 1) {
    *FV = K(0.0);
    *MOZ = K(0.0);
    MOL = K(0.0);
    MOZ2 = K(0.0);
  } else {
    real TVIR = (K(1.0) + K(0.61) * QAIR) * SFCTMP;
    real TMP1 = DV(1, KARMAN * DV(0, GRAV, TVIR) * H, (RHOAIR * CPAIR));
    if (FABS(TMP1) <= MPEl) TMP1 = MPEl;
    MOL = DV(2, K(-1.0) * p3(*FV), TMP1);
    *MOZ = rmin(DV(3, (ZLVL - ZPD), MOL), K(1.0));
    MOZ2 = rmin(DV(4, (K(2.0) + Z0H), MOL), K(1.0));
  }
  if (MOZOLD * *MOZ < K(0.0)) *MOZSGN = *MOZSGN + 1;
  if (*MOZSGN >= 2) {
    *MOZ = K(0.0);
    *FM = K(0.0);
    *FH = K(0.0);
    MOZ2 = K(0.0);
    *FM2 = K(0.0);
    *FH2 = K(0.0);
  }
  real FMNEW, FHNEW, FM2NEW, FH2NEW;
  if (*MOZ < K(0.0)) {
    real TMP1 = POW(K(1.0) - K(16.0) * *MOZ, K(0.25));
    real TMP2 = LOG((K(1.0) + TMP1 * TMP1) / K(2.0));
    real TMP3 = LOG((K(1.0) + TMP1) / K(2.0));
    FMNEW = K(2.0) * TMP3 + TMP2 - K(2.0) * ATAN(TMP1) + K(1.5707963);
    FHNEW = K(2.0) * TMP2;
    real TMP12 = POW(K(1.0) - K(16.0) * MOZ2, K(0.25));
    real TMP22 = LOG((K(1.0) + TMP12 * TMP12) / K(2.0));
    real TMP32 = LOG((K(1.0) + TMP12) / K(2.0));
    FM2NEW = K(2.0) * TMP32 + TMP22 - K(2.0) * ATAN(TMP12) + K(1.5707963);
    FH2NEW = K(2.0) * TMP22;
  } else {
    FMNEW = K(-5.0) * *MOZ;
    FHNEW = FMNEW;
    FM2NEW = K(-5.0) * MOZ2;
    FH2NEW = FM2NEW;
  }
  if (iter == 1) {
    *FM = FMNEW;
    *FH = FHNEW;
    *FM2 = FM2NEW;
    *FH2 = FH2NEW;
  } else {
    *FM = K(0.5) * (*FM + FMNEW);
    *FH = K(0.5) * (*FH + FHNEW);
    *FM2 = K(0.5) * (*FM2 + FM2NEW);
    *FH2 = K(0.5) * (*FH2 + FH2NEW);
  }
  *FH = rmin(*FH, K(0.9) * TMPCH);
  *FM = rmin(*FM, K(0.9) * TMPCM);
  *FH2 = rmin(*FH2, K(0.9) * TMPCH2);
  *FM2 = rmin(*FM2, K(0.9) * TMPCM2);
  real CMFM = TMPCM - *FM;
  real CHFH = TMPCH - *FH;
  real CM2FM2 = TMPCM2 - *FM2;
  real CH2FH2 = TMPCH2 - *FH2;
  if (FABS(CMFM) <= MPEl) CMFM = MPEl;
  if (FABS(CHFH) <= MPEl) CHFH = MPEl;
  if (FABS(CM2FM2) <= MPEl) CM2FM2 = MPEl;
  if (FABS(CH2FH2) <= MPEl) CH2FH2 = MPEl;
  *CM = DV(5, KARMAN * KARMAN, (CMFM * CMFM));
  *CH = DV(6, KARMAN * KARMAN, (CMFM * CHFH));
  *CH2 = KARMAN * KARMAN / (CM2FM2 * CH2FH2);
  *FV = UR * SQRT(*CM);
  *CH2 = KARMAN * *FV / CH2FH2;
}

/* sfcdif2: func.f90:3511-3689 (Chen97, opt_sfc=2) */
static void sfcdif2(int iter, real Z0, real THZ0, real THLM, real SFCSPD, real CZIL, real ZLM,
                    real* AKMS, real* AKHS, real* RLMO, real* WSTAR2, real* USTAR) {
  const real WWST = K(1.2);
  const real WWST2 = WWST * WWST;
  const real VKRM = K(0.40), EXCM = K(0.001);
  const real BETA = K(1.0) / K(270.0);
  const real BTG = BETA * GRAV;
  const real ELFC = VKRM * BTG;
  const real WOLD = K(0.15);
  const real WNEW = K(1.0) - WOLD;
  const real PIHF = K(3.14159265) / K(2.);
  const real EPSU2 = K(1.E-4), EPSUST = K(0.07), ZTMIN = K(-5.0), ZTMAX = K(1.0);
  const real HPBL = K(1000.0), SQVISC = K(258.2);
  real ZILFC = -CZIL * VKRM * SQVISC;
  real ZU = Z0;
  real RDZ = K(1.0) / ZLM;
  real CXCH = EXCM * RDZ;
  real DTHV = THLM - THZ0;
  real DU2 = rmax(SFCSPD * SFCSPD, EPSU2);
  real BTGH = BTG * HPBL;
  if (iter == 1) {
    if (BTGH * *AKHS * DTHV != K(0.0))
      *WSTAR2 = WWST2 * POW(FABS(BTGH * *AKHS * DTHV), K(2.0) / K(3.0));
    else
      *WSTAR2 = K(0.0);
    *USTAR = rmax(SQRT(*AKMS * SQRT(DU2 + *WSTAR2)), EPSUST);
    *RLMO = ELFC * *AKHS * DTHV / p3(*USTAR);
  }
  real ZT = rmax(K(1.0E-6), EXP(ZILFC * SQRT(*USTAR * Z0)) * Z0);
  real ZSLU = ZLM + ZU;
  real ZSLT = ZLM + ZT;
  real RLOGU = LOG(ZSLU / ZU);
  real RLOGT = LOG(ZSLT / ZT);
  real ZETALT = rmax(ZSLT * *RLMO, ZTMIN);
  *RLMO = ZETALT / ZSLT;
  real ZETALU = ZSLU * *RLMO;
  real ZETAU = ZU * *RLMO;
  real ZETAT = ZT * *RLMO;
  real SIMM, SIMH;
#define PSPMU(XX) (K(-2.0) * LOG(((XX) + K(1.0)) * K(0.5)) - LOG(((XX) * (XX) + K(1.0)) * K(0.5)) + \
                   K(2.0) * ATAN(XX) - PIHF)
#define PSPHU(XX) (K(-2.0) * LOG(((XX) * (XX) + K(1.0)) * K(0.5)))
  if (*RLMO < K(0.0)) {
    real XLU4 = K(1.0) - K(16.0) * ZETALU;
    real XLT4 = K(1.0) - K(16.0) * ZETALT;
    real XU4 = K(1.0) - K(16.0) * ZETAU;
    real XT4 = K(1.0) - K(16.0) * ZETAT;
    real XLU = SQRT(SQRT(XLU4)), XLT = SQRT(SQRT(XLT4)), XU = SQRT(SQRT(XU4));
    real XT = SQRT(SQRT(XT4));
    real PSMZ = PSPMU(XU);
    SIMM = PSPMU(XLU) - PSMZ + RLOGU;
    real PSHZ = PSPHU(XT);
    SIMH = PSPHU(XLT) - PSHZ + RLOGT;
  } else {
    ZETALU = rmin(ZETALU, ZTMAX);
    ZETALT = rmin(ZETALT, ZTMAX);
    real PSMZ = K(5.0) * ZETAU;
    SIMM = K(5.0) * ZETALU - PSMZ + RLOGU;
    real PSHZ = K(5.0) * ZETAT;
    SIMH = K(5.0) * ZETALT - PSHZ + RLOGT;
  }
#undef PSPMU
#undef PSPHU
  *USTAR = rmax(SQRT(*AKMS * SQRT(DU2 + *WSTAR2)), EPSUST);
  ZT = rmax(K(1.E-6), EXP(ZILFC * SQRT(*USTAR * Z0)) * Z0);
  ZSLT = ZLM + ZT;
  RLOGT = LOG(ZSLT / ZT);
  real USTARK = *USTAR * VKRM;
  *AKMS = rmax(USTARK / SIMM, CXCH);
  *AKHS = rmax(USTARK / SIMH, CXCH);
  if (BTGH * *AKHS * DTHV != K(0.0))
    *WSTAR2 = WWST2 * POW(FABS(BTGH * *AKHS * DTHV), K(2.0) / K(3.0));
  else
    *WSTAR2 = K(0.0);
  real RLMN = ELFC * *AKHS * DTHV / p3(*USTAR);
  real RLMA = *RLMO * WOLD + RLMN * WNEW;
  *RLMO = RLMA;
}

/* ragrb: func.f90:3260-3350 */
static void ragrb(const nmp_params* P, int iter, real VAI, real RHOAIR, real HG, real TAH,
                  real ZPD, real Z0MG, real Z0HG, real HCAN, real UC, real Z0H, real FV, real CWP,
                  int lutyp, real MPEl, real* MOZG, real* FHG, real* RAMG, real* RAHG, real* RAWG,
                  real* RB) {
  *MOZG = K(0.0);
  real MOLG = K(0.0);
  if (iter > 1) {
    real TMP1 = DV(11, KARMAN * DV(10, GRAV, TAH) * HG, (RHOAIR * CPAIR));
    if (FABS(TMP1) <= MPEl) TMP1 = MPEl;
    MOLG = DV(12, K(-1.) * p3(FV), TMP1);
    *MOZG = rmin(DV(13, (ZPD - Z0MG), MOLG), K(1.0));
  }
  real FHGNEW = (*MOZG < K(0.0)) ? POW(K(1.0) - K(15.0) * *MOZG, K(-0.25))
                                  : K(1.0) + K(4.7) * *MOZG;
  if (iter == 1)
    *FHG = FHGNEW;
  else
    *FHG = K(0.5) * (*FHG + FHGNEW);
  real CWPC = SQRT(CWP * VAI * HCAN * *FHG);
  real TMP1 = EXP(DV(14, -CWPC * Z0HG, HCAN));
  real TMP2 = EXP(DV(15, -CWPC * (Z0H + ZPD), HCAN));
  real TMPRAH2 = DV(16, HCAN * EXP(CWPC), CWPC) * (TMP1 - TMP2);
  real KH = rmax(KARMAN * FV * (HCAN - ZPD), MPEl);
  *RAMG = K(0.0);
  *RAHG = DV(17, TMPRAH2, KH);
  *RAWG = *RAHG;
  real TMPRB = DV(18, CWPC * K(50.0), (K(1.0) - EXP(-CWPC / K(2.0))));
  *RB = TMPRB * SQRT(VEGP(dleaf) / UC);
}

/* stomata (Ball-Berry, this repo's bisection variant): func.f90:3739-3887 */
static void stomata(const nmp_params* P, int lutyp, real igs, real sfcprs, real sfctmp, real apar,
                    real tv, real ea, real ei, real o2, real co2, real foln, real btran, real rb,
                    real* rs, real* psn) {
  const real CIERR = K(5.0E-2);
  real cf = sfcprs / (RGAS * sfctmp) * K(1.0e06);
  *rs = K(1.0) / VEGP(bp) * cf;
  *psn = K(0.0);
  if (apar <= K(0.0)) return;
  real fnf = rmin(foln / rmax(MPE, VEGP(folnmx)), K(1.0));
  real tc = tv - TFRZ;
  real ppf = K(4.6) * apar;
  real j = ppf * VEGP(qe25);
  real kc = VEGP(kc25) * POW(VEGP(akc), (tc - K(25.0)) / K(10.0));
  real ko = VEGP(ko25) * POW(VEGP(ako), (tc - K(25.0)) / K(10.0));
  real awc = kc * (K(1.0) + o2 / ko);
  real cp = K(0.5) * kc / ko * o2 * K(0.21);
  real vcmx = VEGP(vcmx25) /
              (K(1.0) + EXP((K(-2.2E05) + K(710.0) * (tc + TFRZ)) / (K(8.314) * (tc + TFRZ)))) *
              fnf * btran * (POW(VEGP(avcmx), (tc - K(25.0)) / K(10.0)));
  real rlb = rb / cf;
  real cihigh = K(1.5) * co2, cilow = K(0.0);
  const int c3c4 = P->c3c4[lutyp - 1];
  for (int iter = 1; iter <= 20; ++iter) { ITER_STAT(1);
    real ci = K(0.5) * (cihigh + cilow);
    /* ci2ci: func.f90:3847-3886.  The reference keeps wc/wj/we SAVEd (nan4
     * initialised); for C3C4 outside {1,2} we use that initial NaN. */
    real wc = NAN, wj = NAN, we = NAN;
    if (c3c4 == 1) {
      wj = rmax(ci - cp, K(0.0)) * j / (ci + K(2.0) * cp);
      wc = rmax(ci - cp, K(0.0)) * vcmx / (ci + awc);
      we = K(0.5) * vcmx;
    } else if (c3c4 == 2) {
      wj = j;
      wc = vcmx;
      we = K(4000.0) * vcmx * ci / sfcprs;
    }
    *psn = rmin(rmin(wj, wc), we) * igs;
    real cs = rmax(co2 - K(1.37) * rlb * sfcprs * *psn, MPE);
    real a = VEGP(mp) * *psn * sfcprs * ea / (cs * ei) + VEGP(bp);
    real b = (VEGP(mp) * *psn * sfcprs / cs + VEGP(bp)) * rlb - K(1.0);
    real c = -rlb;
    real q;
    if (b >= K(0.0))
      q = K(-0.5) * (b + SQRT(b * b - K(4.0) * a * c));
    else
      q = K(-0.5) * (b - SQRT(b * b - K(4.0) * a * c));
    real r1 = q / a;
    real r2 = c / q;
    *rs = rmax(r1, r2);
    real fci = rmax(cs - *psn * sfcprs * K(1.65) * *rs, K(0.0));
    if (((cihigh - cilow) <= CIERR) || FABS(fci - ci) <= MPE) break;
    if (fci > ci)
      cilow = ci;
    else
      cihigh = ci;
  }
  *rs = *rs * cf;
}

/* calhum: func.f90:3958-3984 */
static void calhum(real SFCTMP, real SFCPRS, real* Q2SAT, real* DQSDT2) {
  const real A2 = K(17.67), A3 = K(273.15), A4 = K(29.65), ELWV = K(2.501E6);
  const real A23M4 = A2 * (A3 - A4), E0 = K(0.611), RV = K(461.0), EPSILON = K(0.622);
  real ES = E0 * EXP(ELWV / RV * (K(1.) / A3 - K(1.) / SFCTMP));
  real SFCPRSX = SFCPRS * K(1.E-3);
  *Q2SAT = EPSILON * ES / (SFCPRSX - ES);
  *Q2SAT = *Q2SAT * K(1.E3);
  *DQSDT2 = (*Q2SAT / (1 + *Q2SAT)) * A23M4 / p2(SFCTMP - A4);
  *Q2SAT = *Q2SAT / K(1.E3);
}

/* canres (Jarvis, opt_crs=2): func.f90:3890-3955 -- psn = NaN as in the reference */
static void canres(const nmp_params* P, int lutyp, real sfcprs, real tv, real par, real eah,
                   real btran, real* rs, real* psn) {
  real q2 = K(0.622) * eah / (sfcprs - K(0.378) * eah);
  q2 = q2 / (K(1.0) + q2);
  real q2sat, dqsdt2;
  calhum(tv, sfcprs, &q2sat, &dqsdt2);
  real ff = K(2.0) * par / VEGP(rgl);
  real rcs = (ff + VEGP(rsmin) / VEGP(rsmax)) / (K(1.0) + ff);
  rcs = rmin(rmax(rcs, K(0.0001)), K(1.0));
  real rct = K(1.0) - K(0.0016) * p2(VEGP(topt) - tv);
  rct = rmin(rmax(rct, K(0.0001)), K(1.0));
  real rcq = K(1.0) / (K(1.0) + VEGP(hs) * rmax(K(0.0), q2sat - q2));
  rcq = rmin(rmax(rcq, K(0.01)), K(1.0));
  *rs = VEGP(rsmin) / (rcs * rct * rcq * btran);
  *psn = NAN;
}

typedef struct { /* vege_flux outputs (func.f90:2570-2586) */
  real TAUXV, TAUYV, IRG, IRC, SHG, SHC, EVG, EVC, TR, GH, T2MV, PSNSUN, PSNSHA, Q2V, CAH2,
      CHLEAF, CHUC, RSSUN, RSSHA;
} vegout_t;

/* vege_flux: func.f90:2465-2964 */
static void vege_flux(ctx_t* X, int ISNOW, int lutyp, real DT, real SAV, real SAG, real LWDN,
                      real UR, real UU, real VV, real SFCTMP, real THAIR, real QAIR, real EAIR,
                      real RHOAIR, real snowh, real VAI, real GAMMAV, real GAMMAG, real FWET,
                      real LAISUN, real LAISHA, real CWP, const real* DZSNSO, real HTOP,
                      real ZLVL, real ZPD, real Z0M, real fveg, real Z0MG, real EMV, real EMG,
                      real CANLIQ, real CANICE, const real* STC, const real* DF, real RSURF,
                      real LATHEAV, real LATHEAG, real PARSUN, real PARSHA, real IGS, real FOLN,
                      real CO2AIR, real O2AIR, real BTRAN, real SFCPRS, real RHSUR, real PSFC,
                      real* EAH, real* TAH, real* TV, real* TG, real* CM, real* CH, real* QSFC,
                      vegout_t* o) {
  const nmp_params* P = X->P;
  const int NITERC = 20, NITERG = 5;
  real MPEl = K(1E-6);
  int LITER = 0;
  real FV = K(0.1);
  real DTV = K(0.0), DTG = K(0.0);
  int MOZSGN = 0;
  real HG = K(0.0), H = K(0.0);
  real MOZ = K(0.0), FM = K(0.0), FH = K(0.0), FM2 = K(0.0), FH2 = K(0.0), CH2 = K(0.0);
  real MOZG = K(0.0), FHG = K(0.0), WSTAR = K(0.0);
  real RAMC, RAHC, RAWC, RAMG = K(0.0), RAHG = K(0.0), RAWG = K(0.0), RB = K(0.0);
  real CAH = K(0.0), CVH = K(0.0), CGH, COND, ATA, BTA, CSH, CAW, CEW, CTW, CGW, AEA, BEA, CEV, CTR;
  real ESTV, DESTV = K(0.0), ESTG, DESTG, ESATW, ESATI, DSATW, DSATI, A, B, T;
  real Z0H = Z0M, Z0HG = Z0MG;

  real VAIE = rmin(K(6.0), VAI / fveg);
  real LAISUNE = rmin(K(6.0), LAISUN / fveg);
  real LAISHAE = rmin(K(6.0), LAISHA / fveg);

  T = tdc(*TG);
  esat(T, &ESATW, &ESATI, &DSATW, &DSATI);
  ESTG = (T > K(0.0)) ? ESATW : ESATI;

  *QSFC = K(0.622) * EAIR / (PSFC - K(0.378) * EAIR);

  real HCAN = HTOP;
  real UC = UR * LOG(HCAN / Z0M) / LOG(ZLVL / Z0M);
  if ((HCAN - ZPD) <= K(0.0)) X->status |= NMP_ST_HCAN;

  real AIR = -EMV * (K(1.0) + (K(1.0) - EMV) * (K(1.0) - EMG)) * LWDN - EMV * EMG * SB * p4(*TG);
  real CIR = (K(2.0) - EMV * (K(1.0) - EMG)) * EMV * SB;

  for (int iter = 1; iter <= NITERC; ++iter) { ITER_STAT(0);
    Z0H = Z0M;
    Z0HG = Z0MG;
    if (X->O->opt_sfc == 1)
      sfcdif1(X, iter, SFCTMP, RHOAIR, H, QAIR, ZLVL, ZPD, Z0M, Z0H, UR, MPEl, &MOZ, &MOZSGN, &FM,
              &FH, &FM2, &FH2, CM, CH, &FV, &CH2);
    if (X->O->opt_sfc == 2) {
      sfcdif2(iter, Z0M, *TAH, THAIR, UR, (real)P->czil, ZLVL, CM, CH, &MOZ, &WSTAR, &FV);
      *CH = *CH / UR;
      *CM = *CM / UR;
    }
    RAMC = rmax(K(1.0), K(1.0) / (*CM * UR));
    RAHC = rmax(K(1.0), DV(7, K(1.0), (*CH * UR)));
    RAWC = RAHC;
    ragrb(P, iter, VAIE, RHOAIR, HG, *TAH, ZPD, Z0MG, Z0HG, HCAN, UC, Z0H, FV, CWP, lutyp, MPEl,
          &MOZG, &FHG, &RAMG, &RAHG, &RAWG, &RB);
    T = tdc(*TV);
    esat(T, &ESATW, &ESATI, &DSATW, &DSATI);
    if (T > K(0.0)) {
      ESTV = ESATW;
      DESTV = DSATW;
    } else {
      ESTV = ESATI;
      DESTV = DSATI;
    }
    if (iter == 1) {
      if (X->O->opt_crs == 1) {
        stomata(P, lutyp, IGS, SFCPRS, SFCTMP, PARSUN, *TV, *EAH, ESTV, O2AIR, CO2AIR, FOLN,
                BTRAN, RB, &o->RSSUN, &o->PSNSUN);
        stomata(P, lutyp, IGS, SFCPRS, SFCTMP, PARSHA, *TV, *EAH, ESTV, O2AIR, CO2AIR, FOLN,
                BTRAN, RB, &o->RSSHA, &o->PSNSHA);
      }
      if (X->O->opt_crs == 2) {
        canres(P, lutyp, SFCPRS, *TV, PARSUN, *EAH, BTRAN, &o->RSSUN, &o->PSNSUN);
        canres(P, lutyp, SFCPRS, *TV, PARSHA, *EAH, BTRAN, &o->RSSHA, &o->PSNSHA);
      }
    }
    CAH = DV(20, K(1.0), RAHC);
    CVH = DV(21, K(2.0) * VAIE, RB);
    CGH = DV(22, K(1.0), RAHG);
    COND = CAH + CVH + CGH;
    ATA = DV(23, (SFCTMP * CAH + *TG * CGH), COND);
    BTA = DV(24, CVH, COND);
    CSH = (K(1.0) - BTA) * RHOAIR * CPAIR * CVH;
    CAW = DV(25, K(1.0), RAWC);
    CEW = DV(26, FWET * VAIE, RB);
    CTW = (K(1.0) - FWET) * (DV(27, LAISUNE, (RB + o->RSSUN)) + DV(28, LAISHAE, (RB + o->RSSHA)));
    CGW = DV(29, K(1.0), (RAWG + RSURF));
    COND = CAW + CEW + CTW + CGW;
    AEA = DV(30, (EAIR * CAW + ESTG * CGW), COND);
    BEA = DV(31, (CEW + CTW), COND);
    CEV = DV(32, (K(1.0) - BEA) * CEW * RHOAIR * CPAIR, GAMMAV);
    CTR = DV(33, (K(1.0) - BEA) * CTW * RHOAIR * CPAIR, GAMMAV);
    *TAH = ATA + BTA * *TV;
    *EAH = AEA + BEA * ESTV;
    o->IRC = fveg * (AIR + CIR * p4(*TV));
    o->SHC = fveg * RHOAIR * CPAIR * CVH * (*TV - *TAH);
    o->EVC = DV(34, fveg * RHOAIR * CPAIR * CEW * (ESTV - *EAH), GAMMAV);
    o->TR = DV(35, fveg * RHOAIR * CPAIR * CTW * (ESTV - *EAH), GAMMAV);
    if (*TV > TFRZ)
      o->EVC = rmin(CANLIQ * LATHEAV / DT, o->EVC);
    else
      o->EVC = rmin(CANICE * LATHEAV / DT, o->EVC);
    B = SAV - o->IRC - o->SHC - o->EVC - o->TR;
    A = fveg * (K(4.0) * CIR * p3(*TV) + CSH + (CEV + CTR) * DESTV);
    DTV = DV(36, B, A);
    o->IRC = o->IRC + fveg * K(4.0) * CIR * p3(*TV) * DTV;
    o->SHC = o->SHC + fveg * CSH * DTV;
    o->EVC = o->EVC + fveg * CEV * DESTV * DTV;
    o->TR = o->TR + fveg * CTR * DESTV * DTV;
    *TV = *TV + DTV;
    H = DV(37, RHOAIR * CPAIR * (*TAH - SFCTMP), RAHC);
    HG = DV(38, RHOAIR * CPAIR * (*TG - *TAH), RAHG);
    *QSFC = DV(39, (K(0.622) * *EAH), (SFCPRS - K(0.378) * *EAH));
    if (LITER == 1) break;
    if (iter >= 5 && FABS(DTV) <= K(0.01) && LITER == 0) LITER = 1;
  }

  AIR = -EMG * (K(1.0) - EMV) * LWDN - EMG * EMV * SB * p4(*TV);
  CIR = EMG * SB;
  CSH = RHOAIR * CPAIR / RAHG;
  CEV = RHOAIR * CPAIR / (GAMMAG * (RAWG + RSURF));
  CGH = K(2.0) * DF[ISNOW + 1] / DZSNSO[ISNOW + 1];
  ESTG = K(0.0);
  for (int iter = 1; iter <= NITERG; ++iter) { ITER_STAT(4);
    T = tdc(*TG);
    esat(T, &ESATW, &ESATI, &DSATW, &DSATI);
    if (T > K(0.0)) {
      ESTG = ESATW;
      DESTG = DSATW;
    } else {
      ESTG = ESATI;
      DESTG = DSATI;
    }
    o->IRG = CIR * p4(*TG) + AIR;
    o->SHG = CSH * (*TG - *TAH);
    o->EVG = CEV * (ESTG * RHSUR - *EAH);
    o->GH = CGH * (*TG - STC[ISNOW + 1]);
    B = SAG - o->IRG - o->SHG - o->EVG - o->GH;
    A = K(4.0) * CIR * p3(*TG) + CSH + CEV * DESTG + CGH;
    DTG = B / A;
    o->IRG = o->IRG + K(4.0) * CIR * p3(*TG) * DTG;
    o->SHG = o->SHG + CSH * DTG;
    o->EVG = o->EVG + CEV * DESTG * DTG;
    o->GH = o->GH + CGH * DTG;
    *TG = *TG + DTG;
  }
  if (X->O->opt_stc == 1) {
    if (snowh > K(0.05) && *TG > TFRZ) {
      *TG = TFRZ;
      o->IRG = CIR * p4(*TG) - EMG * (K(1.0) - EMV) * LWDN - EMG * EMV * SB * p4(*TV);
      o->SHG = CSH * (*TG - *TAH);
      o->EVG = CEV * (ESTG * RHSUR - *EAH);
      o->GH = SAG - (o->IRG + o->SHG + o->EVG);
    }
  }
  o->TAUXV = -RHOAIR * *CM * UR * UU;
  o->TAUYV = -RHOAIR * *CM * UR * VV;
  if (X->O->opt_sfc == 1 || X->O->opt_sfc == 2) {
    o->CAH2 = FV * KARMAN / (LOG((K(2.0) + Z0H) / Z0H) - FH2);
    real CQ2V = o->CAH2;
    if (o->CAH2 < K(1.E-5)) {
      o->T2MV = *TAH;
      o->Q2V = *QSFC;
    } else {
      o->T2MV = *TAH - (o->SHG + o->SHC / fveg) / (RHOAIR * CPAIR) * K(1.0) / o->CAH2;
      o->Q2V = *QSFC - ((o->EVC + o->TR) / fveg + o->EVG) / (LATHEAV * RHOAIR) * K(1.0) / CQ2V;
    }
  }
  *CH = CAH;
  o->CHLEAF = CVH;
  o->CHUC = K(1.0) / RAHG;
}

typedef struct { /* bare_flux outputs (func.f90:3038-3050) */
  real TAUXB, TAUYB, IRB, SHB, EVB, GHB, T2MB, Q2B, EHB2;
} bareout_t;

/* bare_flux: func.f90:2967-3257 */
static void bare_flux(ctx_t* X, int lutyp, int ISNOW, real SAG, real LWDN, real UR, real UU,
                      real VV, real SFCTMP, real THAIR, real QAIR, real EAIR, real RHOAIR,
                      real snowh, const real* DZSNSO, real ZLVL, real ZPD, real Z0M, real EMG,
                      const real* STC, const real* DF, real RSURF, real LATHEA, real GAMMA,
                      real RHSUR, real PSFC, real* TGB, real* CM, real* CH, real* QSFC,
                      bareout_t* o) {
  const nmp_params* P = X->P;
  real MPEl = K(1.0E-6);
  real DTG = K(0.0);
  int MOZSGN = 0;
  real H = K(0.0), FV = K(0.1);
  real MOZ = K(0.0), FM = K(0.0), FH = K(0.0), FM2 = K(0.0), FH2 = K(0.0), CH2 = K(0.0),
       WSTAR = K(0.0);
  real CIR = EMG * SB;
  real CGH = K(2.0) * DF[ISNOW + 1] / DZSNSO[ISNOW + 1];
  real Z0H = Z0M, RAMB, RAHB, RAWB, EHB = K(0.0), CSH = K(0.0), CEV = K(0.0), A, B, T;
  real ESTG = K(0.0), DESTG, ESATW, ESATI, DSATW, DSATI;
  for (int iter = 1; iter <= 5; ++iter) {
    Z0H = Z0M;
    if (X->O->opt_sfc == 1)
      sfcdif1(X, iter, SFCTMP, RHOAIR, H, QAIR, ZLVL, ZPD, Z0M, Z0H, UR, MPEl, &MOZ, &MOZSGN, &FM,
              &FH, &FM2, &FH2, CM, CH, &FV, &CH2);
    if (X->O->opt_sfc == 2) {
      sfcdif2(iter, Z0M, *TGB, THAIR, UR, (real)P->czil, ZLVL, CM, CH, &MOZ, &WSTAR, &FV);
      *CH = *CH / UR;
      *CM = *CM / UR;
      if (snowh > K(0.0)) {
        *CM = rmin(K(0.01), *CM);
        *CH = rmin(K(0.01), *CH);
      }
    }
    RAMB = rmax(K(1.0), K(1.0) / (*CM * UR));
    RAHB = rmax(K(1.0), K(1.0) / (*CH * UR));
    RAWB = RAHB;
    EHB = K(1.0) / RAHB;
    T = tdc(*TGB);
    esat(T, &ESATW, &ESATI, &DSATW, &DSATI);
    if (T > K(0.0)) {
      ESTG = ESATW;
      DESTG = DSATW;
    } else {
      ESTG = ESATI;
      DESTG = DSATI;
    }
    CSH = RHOAIR * CPAIR / RAHB;
    CEV = RHOAIR * CPAIR / GAMMA / (RSURF + RAWB);
    o->IRB = CIR * p4(*TGB) - EMG * LWDN;
    o->SHB = CSH * (*TGB - SFCTMP);
    o->EVB = CEV * (ESTG * RHSUR - EAIR);
    o->GHB = CGH * (*TGB - STC[ISNOW + 1]);
    B = SAG - o->IRB - o->SHB - o->EVB - o->GHB;
    A = K(4.0) * CIR * p3(*TGB) + CSH + CEV * DESTG + CGH;
    DTG = B / A;
    o->IRB = o->IRB + K(4.0) * CIR * p3(*TGB) * DTG;
    o->SHB = o->SHB + CSH * DTG;
    o->EVB = o->EVB + CEV * DESTG * DTG;
    o->GHB = o->GHB + CGH * DTG;
    *TGB = *TGB + DTG;
    H = CSH * (*TGB - SFCTMP);
    T = tdc(*TGB);
    esat(T, &ESATW, &ESATI, &DSATW, &DSATI);
    ESTG = (T > K(0.0)) ? ESATW : ESATI;
    *QSFC = K(0.622) * (ESTG * RHSUR) / (PSFC - K(0.378) * (ESTG * RHSUR));
  }
  if (X->O->opt_stc == 1) {
    if (snowh > K(0.05) && *TGB > TFRZ) {
      *TGB = TFRZ;
      o->IRB = CIR * p4(*TGB) - EMG * LWDN;
      o->SHB = CSH * (*TGB - SFCTMP);
      o->EVB = CEV * (ESTG * RHSUR - EAIR);
      o->GHB = SAG - (o->IRB + o->SHB + o->EVB);
    }
  }
  o->TAUXB = -RHOAIR * *CM * UR * UU;
  o->TAUYB = -RHOAIR * *CM * UR * VV;
  if (X->O->opt_sfc == 1 || X->O->opt_sfc == 2) {
    o->EHB2 = FV * KARMAN / (LOG((K(2.0) + Z0H) / Z0H) - FH2);
    real CQ2B = o->EHB2;
    if (o->EHB2 < K(1.0E-5)) {
      o->T2MB = *TGB;
      o->Q2B = *QSFC;
    } else {
      o->T2MB = *TGB - o->SHB / (RHOAIR * CPAIR) * K(1.0) / o->EHB2;
      o->Q2B = *QSFC - o->EVB / (LATHEA * RHOAIR) * (K(1.0) / CQ2B + RSURF);
    }
    if (lutyp == P->isurban) o->Q2B = *QSFC;
  }
  *CH = EHB;
}

/* rosr12: func.f90:4240-4288 (arrays indexed NTOP..NSOIL) */
static void rosr12(real* Pp, const real* A, const real* B, real* C, const real* D, real* DELTA,
                   int NTOP, int NSOILl) {
  C[NSOILl] = K(0.0);
  Pp[NTOP] = -C[NTOP] / B[NTOP];
  DELTA[NTOP] = D[NTOP] / B[NTOP];
  for (int k = NTOP + 1; k <= NSOILl; ++k) {
    Pp[k] = -C[k] * (K(1.0) / (B[k] + A[k] * Pp[k - 1]));
    DELTA[k] = (D[k] - A[k] * DELTA[k - 1]) * (K(1.0) / (B[k] + A[k] * Pp[k - 1]));
  }
  Pp[NSOILl] = DELTA[NSOILl];
  for (int k = NTOP + 1; k <= NSOILl; ++k) {
    int kk = NSOILl - k + (NTOP - 1) + 1;
    Pp[kk] = Pp[kk] * Pp[kk + 1] + DELTA[kk];
  }
}

/* tsnosoi + hrt + hstep: func.f90:3987-4237 */
static void tsnosoi(ctx_t* X, int ISNOW, real TBOT, const real* ZSNSO, real SSOIL, const real* DF,
                    const real* HCPCT, real ZBOT, real DT, real snowh, real* STC) {
  real AIb[7] = {0}, BIb[7] = {0}, CIb[7] = {0}, RHSb[7] = {0}, DDZb[7], DENOMb[7], DTSDZb[7], EFLUXb[7], CIINb[7],
      RHSINb[7] = {0};
  real *AI = AIb + 2, *BI = BIb + 2, *CI = CIb + 2, *RHSTS = RHSb + 2, *DDZ = DDZb + 2,
       *DENOM = DENOMb + 2, *DTSDZ = DTSDZb + 2, *EFLUX = EFLUXb + 2, *CIIN = CIINb + 2,
       *RHSTSIN = RHSINb + 2;
  const int otb = X->O->opt_tbot, ostc = X->O->opt_stc;
  real ZBOTSNO = ZBOT - snowh;
  real BOTFLX = K(0.0), TEMP1;
  /* hrt: func.f90:4099-4188 (PHI = 0) */
  for (int k = ISNOW + 1; k <= NSOIL; ++k) {
    if (k == ISNOW + 1) {
      DENOM[k] = -ZSNSO[k] * HCPCT[k];
      TEMP1 = -ZSNSO[k + 1];
      DDZ[k] = K(2.0) / TEMP1;
      DTSDZ[k] = K(2.0) * (STC[k] - STC[k + 1]) / TEMP1;
      EFLUX[k] = DF[k] * DTSDZ[k] - SSOIL - K(0.0);
    } else if (k < NSOIL) {
      DENOM[k] = (ZSNSO[k - 1] - ZSNSO[k]) * HCPCT[k];
      TEMP1 = ZSNSO[k - 1] - ZSNSO[k + 1];
      DDZ[k] = K(2.0) / TEMP1;
      DTSDZ[k] = K(2.0) * (STC[k] - STC[k + 1]) / TEMP1;
      EFLUX[k] = (DF[k] * DTSDZ[k] - DF[k - 1] * DTSDZ[k - 1]) - K(0.0);
    } else {
      DENOM[k] = (ZSNSO[k - 1] - ZSNSO[k]) * HCPCT[k];
      if (otb == 1) BOTFLX = K(0.);
      if (otb == 2) {
        DTSDZ[k] = (STC[k] - TBOT) / (K(0.5) * (ZSNSO[k - 1] + ZSNSO[k]) - ZBOTSNO);
        BOTFLX = -DF[k] * DTSDZ[k];
      }
      EFLUX[k] = (-BOTFLX - DF[k - 1] * DTSDZ[k - 1]) - K(0.0);
    }
  }
  for (int k = ISNOW + 1; k <= NSOIL; ++k) {
    if (k == ISNOW + 1) {
      AI[k] = K(0.0);
      CI[k] = -DF[k] * DDZ[k] / DENOM[k];
      if (ostc == 1) BI[k] = -CI[k];
      if (ostc == 2) BI[k] = -CI[k] + DF[k] / (K(0.5) * ZSNSO[k] * ZSNSO[k] * HCPCT[k]);
    } else if (k < NSOIL) {
      AI[k] = -DF[k - 1] * DDZ[k - 1] / DENOM[k];
      CI[k] = -DF[k] * DDZ[k] / DENOM[k];
      BI[k] = -(AI[k] + CI[k]);
    } else {
      AI[k] = -DF[k - 1] * DDZ[k - 1] / DENOM[k];
      CI[k] = K(0.0);
      BI[k] = -(AI[k] + CI[k]);
    }
    RHSTS[k] = EFLUX[k] / (-DENOM[k]);
  }
  /* hstep: func.f90:4190-4237 */
  for (int k = ISNOW + 1; k <= NSOIL; ++k) {
    RHSTS[k] = RHSTS[k] * DT;
    AI[k] = AI[k] * DT;
    BI[k] = K(1.) + BI[k] * DT;
    CI[k] = CI[k] * DT;
  }
  for (int k = ISNOW + 1; k <= NSOIL; ++k) {
    RHSTSIN[k] = RHSTS[k];
    CIIN[k] = CI[k];
  }
  rosr12(CI, AI, BI, CIIN, RHSTSIN, RHSTS, ISNOW + 1, NSOIL);
  for (int k = ISNOW + 1; k <= NSOIL; ++k) STC[k] = STC[k] + CI[k];
}

/* frh2o (opt_frz=2): func.f90:4494-4598 */
static real frh2o(ctx_t* X, int sltyp, real TKELV, real SMC, real soilwat) {
  const nmp_params* P = X->P;
  const real CK = K(8.0), BLIM = K(5.5), ERROR = K(0.005);
  real BX = SOILP(bexp);
  if (SOILP(bexp) > BLIM) BX = BLIM;
  int NLOG = 0, KCOUNT = 0;
  real FREE;
  if (TKELV > (TFRZ - K(1.0E-3))) {
    FREE = SMC;
  } else {
    real SWL = SMC - soilwat;
    if (SWL > (SMC - K(0.02))) SWL = SMC - K(0.02);
    if (SWL < K(0.0)) SWL = K(0.0);
    while ((NLOG < 10) && (KCOUNT == 0)) { ITER_STAT(2);
      NLOG = NLOG + 1;
      real DF = LOG((SOILP(psisat) * GRAV / HFUS) * p2(K(1.0) + CK * SWL) *
                    POW(SOILP(smcmax) / (SMC - SWL), BX)) -
                LOG(-(TKELV - TFRZ) / TKELV);
      real DENOM = K(2.0) * CK / (K(1.0) + CK * SWL) + BX / (SMC - SWL);
      real SWLK = SWL - DF / DENOM;
      if (SWLK > (SMC - K(0.02))) SWLK = SMC - K(0.02);
      if (SWLK < K(0.0)) SWLK = K(0.0);
      real DSWL = FABS(SWLK - SWL);
      SWL = SWLK;
      if (DSWL <= ERROR) KCOUNT = KCOUNT + 1;
    }
    FREE = SMC - SWL;
    if (KCOUNT == 0) {
      X->status |= NMP_ST_FLERCH;
      real FK = POW((HFUS / (GRAV * (-SOILP(psisat)))) * ((TKELV - TFRZ) / TKELV), K(-1.0) / BX) *
                SOILP(smcmax);
      if (FK < K(0.02)) FK = K(0.02);
      FREE = rmin(FK, SMC);
    }
  }
  return FREE;
}

/* phasechange: func.f90:4291-4491 */
static void phasechange(ctx_t* X, int sltyp, int ISNOW, real DT, const real* FACT,
                        const real* DZSNSO, int IST, real* STC, real* SNICE, real* SNLIQ,
                        real* sneqv, real* snowh, real* SMC, real* soilwat, real* QMELT,
                        int* IMELT, real* PONDING) {
  const nmp_params* P = X->P;
  real HMb[7], XMb[7], WMASS0b[7], WICE0b[7], WLIQ0b[7], MICEb[7], MLIQb[7], SCb[7];
  real *HM = HMb + 2, *XM = XMb + 2, *WMASS0 = WMASS0b + 2, *WICE0 = WICE0b + 2,
       *WLIQ0 = WLIQ0b + 2, *MICE = MICEb + 2, *MLIQ = MLIQb + 2, *SUPERCOOL = SCb + 2;
  *QMELT = K(0.0);
  *PONDING = K(0.0);
  real XMF = K(0.0);
  for (int J = -NSNOW + 1; J <= NSOIL; ++J) SUPERCOOL[J] = K(0.0);
  for (int J = ISNOW + 1; J <= 0; ++J) {
    MICE[J] = SNICE[J];
    MLIQ[J] = SNLIQ[J];
  }
  for (int J = 1; J <= NSOIL; ++J) {
    MLIQ[J] = soilwat[J] * DZSNSO[J] * K(1000.0);
    MICE[J] = (SMC[J] - soilwat[J]) * DZSNSO[J] * K(1000.0);
  }
  for (int J = ISNOW + 1; J <= NSOIL; ++J) {
    IMELT[J] = 0;
    HM[J] = K(0.0);
    XM[J] = K(0.0);
    WICE0[J] = MICE[J];
    WLIQ0[J] = MLIQ[J];
    WMASS0[J] = MICE[J] + MLIQ[J];
  }
  if (IST == 1) {
    for (int J = 1; J <= NSOIL; ++J) {
      if (X->O->opt_frz == 1) {
        if (STC[J] < TFRZ) {
          real SMP = HFUS * (TFRZ - STC[J]) / (GRAV * STC[J]);
          SUPERCOOL[J] = SOILP(smcmax) * POW(SMP / SOILP(psisat), K(-1.0) / SOILP(bexp));
          SUPERCOOL[J] = SUPERCOOL[J] * DZSNSO[J] * K(1000.0);
        }
      }
      if (X->O->opt_frz == 2) {
        SUPERCOOL[J] = frh2o(X, sltyp, STC[J], SMC[J], soilwat[J]);
        SUPERCOOL[J] = SUPERCOOL[J] * DZSNSO[J] * K(1000.0);
      }
    }
  }
  for (int J = ISNOW + 1; J <= NSOIL; ++J) {
    if (MICE[J] > K(0.0) && STC[J] >= TFRZ) IMELT[J] = 1;
    if (MLIQ[J] > SUPERCOOL[J] && STC[J] < TFRZ) IMELT[J] = 2;
    if (ISNOW == 0 && *sneqv > K(0.0) && J == 1) {
      if (STC[J] >= TFRZ) IMELT[J] = 1;
    }
  }
  for (int J = ISNOW + 1; J <= NSOIL; ++J) {
    if (IMELT[J] > 0) {
      HM[J] = (STC[J] - TFRZ) / FACT[J];
      STC[J] = TFRZ;
    }
    if (IMELT[J] == 1 && HM[J] < K(0.0)) {
      HM[J] = K(0.0);
      IMELT[J] = 0;
    }
    if (IMELT[J] == 2 && HM[J] > K(0.0)) {
      HM[J] = K(0.0);
      IMELT[J] = 0;
    }
    XM[J] = HM[J] * DT / HFUS;
  }
  if (ISNOW == 0 && *sneqv > K(0.0) && XM[1] > K(0.0)) {
    real TEMP1 = *sneqv;
    *sneqv = rmax(K(0.0), TEMP1 - XM[1]);
    real PROPOR = *sneqv / TEMP1;
    *snowh = rmax(K(0.0), PROPOR * *snowh);
    real HEATR = HM[1] - HFUS * (TEMP1 - *sneqv) / DT;
    if (HEATR > K(0.0)) {
      XM[1] = HEATR * DT / HFUS;
      HM[1] = HEATR;
    } else {
      XM[1] = K(0.0);
      HM[1] = K(0.0);
    }
    *QMELT = rmax(K(0.0), (TEMP1 - *sneqv)) / DT;
    XMF = HFUS * *QMELT;
    *PONDING = TEMP1 - *sneqv;
  }
  for (int J = ISNOW + 1; J <= NSOIL; ++J) {
    if (IMELT[J] > 0 && FABS(HM[J]) > K(0.0)) {
      real HEATR = K(0.0);
      if (XM[J] > K(0.0)) {
        MICE[J] = rmax(K(0.0), WICE0[J] - XM[J]);
        HEATR = HM[J] - HFUS * (WICE0[J] - MICE[J]) / DT;
      } else if (XM[J] < K(0.0)) {
        if (J <= 0) {
          MICE[J] = rmin(WMASS0[J], WICE0[J] - XM[J]);
        } else {
          if (WMASS0[J] < SUPERCOOL[J]) {
            MICE[J] = K(0.0);
          } else {
            MICE[J] = rmin(WMASS0[J] - SUPERCOOL[J], WICE0[J] - XM[J]);
            MICE[J] = rmax(MICE[J], K(0.0));
          }
        }
        HEATR = HM[J] - HFUS * (WICE0[J] - MICE[J]) / DT;
      }
      MLIQ[J] = rmax(K(0.0), WMASS0[J] - MICE[J]);
      if (FABS(HEATR) > K(0.0)) {
        STC[J] = STC[J] + FACT[J] * HEATR;
        if (J <= 0) {
          if (MLIQ[J] * MICE[J] > K(0.0)) STC[J] = TFRZ;
        }
      }
      XMF = XMF + HFUS * (WICE0[J] - MICE[J]) / DT;
      if (J < 1) *QMELT = *QMELT + rmax(K(0.0), (WICE0[J] - MICE[J])) / DT;
    }
  }
  for (int J = ISNOW + 1; J <= 0; ++J) {
    SNLIQ[J] = MLIQ[J];
    SNICE[J] = MICE[J];
  }
  for (int J = 1; J <= NSOIL; ++J) {
    soilwat[J] = MLIQ[J] / (K(1000.0) * DZSNSO[J]);
    SMC[J] = (MLIQ[J] + MICE[J]) / (K(1000.0) * DZSNSO[J]);
  }
}

/* ------------------------------------------------------------------------ */
/* canwater: func.f90:4807-5046 */
static void canwater(ctx_t* X, int lutyp, real dt, real SFCTMP, real UU, real VV, real FCEV,
                     real FCTR, real QPRECC, real QPRECL, real elai, real esai, int IST, real TG,
                     real fveg, int FROZEN_CANOPY, real* CANLIQ, real* CANICE, real* TV,
                     real* CMC, real* ECAN, real* ETRAN, real* QRAIN, real* QSNOW, real* snowhin,
                     real* FWET, real* FPICE) {
  const nmp_params* P = X->P;
  real FP = K(0.0), QINTR, QDRIPR, QTHROR, QINTS, QDRIPS, QTHROS, QEVAC, QDEWC, QFROC, QSUBC;
  *QRAIN = K(0.0);
  *QSNOW = K(0.0);
  *snowhin = K(0.0);
  *ECAN = K(0.0);
  const int osnf = X->O->opt_snf;
  if (osnf == 1) {
    if (SFCTMP > TFRZ + K(2.5)) {
      *FPICE = K(0.0);
    } else {
      if (SFCTMP <= TFRZ + K(0.5))
        *FPICE = K(1.0);
      else if (SFCTMP <= TFRZ + K(2.0))
        *FPICE = K(1.0) - (K(-54.632) + K(0.2) * SFCTMP);
      else
        *FPICE = K(0.6);
    }
  }
  if (osnf == 2) *FPICE = (SFCTMP >= TFRZ + K(2.2)) ? K(0.) : K(1.0);
  if (osnf == 3) *FPICE = (SFCTMP >= TFRZ) ? K(0.0) : K(1.0);
  real BDFALL = rmin(K(120.0), K(67.92) + K(51.25) * EXP((SFCTMP - TFRZ) / K(2.59)));
  real RAIN = (QPRECC + QPRECL) * (K(1.0) - *FPICE);
  real SNOW = (QPRECC + QPRECL) * *FPICE;
  if (QPRECC + QPRECL > K(0.0)) FP = (QPRECC + QPRECL) / (K(10.0) * QPRECC + QPRECL);
  real MAXLIQ = VEGP(canwmxp) * (elai + esai);
  if ((elai + esai) > K(0.0)) {
    QINTR = fveg * RAIN * FP;
    QINTR = rmin(QINTR, (MAXLIQ - *CANLIQ) / dt * (K(1.0) - EXP(-RAIN * dt / MAXLIQ)));
    QINTR = rmax(QINTR, K(0.0));
    QDRIPR = fveg * RAIN - QINTR;
    QTHROR = (K(1.0) - fveg) * RAIN;
  } else {
    QINTR = K(0.0);
    QDRIPR = K(0.0);
    QTHROR = RAIN;
  }
  if (!FROZEN_CANOPY) {
    *ETRAN = rmax(FCTR / HVAP, K(0.0));
    QEVAC = rmax(FCEV / HVAP, K(0.0));
    QDEWC = FABS(rmin(FCEV / HVAP, K(0.0)));
    QSUBC = K(0.0);
    QFROC = K(0.0);
  } else {
    *ETRAN = rmax(FCTR / HSUB, K(0.0));
    QEVAC = K(0.0);
    QDEWC = K(0.0);
    QSUBC = rmax(FCEV / HSUB, K(0.0));
    QFROC = FABS(rmin(FCEV / HSUB, K(0.0)));
  }
  QEVAC = rmin(*CANLIQ / dt, QEVAC);
  *CANLIQ = rmax(K(0.0), *CANLIQ + (QINTR + QDEWC - QEVAC) * dt);
  if (*CANLIQ <= K(1.0E-6)) *CANLIQ = K(0.0);
  real MAXSNO = K(6.6) * (K(0.27) + K(46.0) / BDFALL) * (elai + esai);
  if ((elai + esai) > K(0.0)) {
    QINTS = fveg * SNOW * FP;
    QINTS = rmin(QINTS, (MAXSNO - *CANICE) / dt * (K(1.0) - EXP(-SNOW * dt / MAXSNO)));
    QINTS = rmax(QINTS, K(0.0));
    real FT = rmax(K(0.0), (*TV - K(270.15)) / K(1.87E5));
    real FV = SQRT(UU * UU + VV * VV) / K(1.56E5);
    QDRIPS = rmax(K(0.0), *CANICE) * (FV + FT);
    QTHROS = (K(1.0) - fveg) * SNOW + (fveg * SNOW - QINTS);
  } else {
    QINTS = K(0.0);
    QDRIPS = K(0.0);
    QTHROS = SNOW;
  }
  QSUBC = rmin(*CANICE / dt, QSUBC);
  *CANICE = rmax(K(0.0), *CANICE + (QINTS - QDRIPS) * dt + (QFROC - QSUBC) * dt);
  if (*CANICE <= K(1.0E-6)) *CANICE = K(0.0);
  if (*CANICE > K(0.0))
    *FWET = rmax(K(0.0), *CANICE) / rmax(MAXSNO, K(1.0E-06));
  else
    *FWET = rmax(K(0.0), *CANLIQ) / rmax(MAXLIQ, K(1.0E-06));
  *FWET = POW(rmin(*FWET, K(1.0)), K(0.667));
  if (*CANICE > K(1.0E-6) && *TV > TFRZ) {
    real QMELTC = rmin(*CANICE / dt, (*TV - TFRZ) * CICE * *CANICE / DENICE / (dt * HFUS));
    *CANICE = rmax(K(0.0), *CANICE - QMELTC * dt);
    *CANLIQ = rmax(K(0.0), *CANLIQ + QMELTC * dt);
    *TV = *FWET * TFRZ + (K(1.0) - *FWET) * *TV;
  }
  if (*CANLIQ > K(1.0E-6) && *TV < TFRZ) {
    real QFRZC = rmin(*CANLIQ / dt, (TFRZ - *TV) * CWAT * *CANLIQ / DENWAT / (dt * HFUS));
    *CANLIQ = rmax(K(0.0), *CANLIQ - QFRZC * dt);
    *CANICE = rmax(K(0.0), *CANICE + QFRZC * dt);
    *TV = *FWET * TFRZ + (K(1.0) - *FWET) * *TV;
  }
  *CMC = *CANLIQ + *CANICE;
  *ECAN = QEVAC + QSUBC - QDEWC - QFROC;
  *QRAIN = QDRIPR + QTHROR;
  *QSNOW = QDRIPS + QTHROS;
  *snowhin = *QSNOW / BDFALL;
  if (IST == 2 && TG > TFRZ) {
    *QSNOW = K(0.0);
    *snowhin = K(0.0);
  }
}

/* snowfall: func.f90:5177-5233 */
static void snowfall(real DT, real QSNOW, real snowhin, real SFCTMP, int* ISNOW, real* snowh,
                     real* DZSNSO, real* STC, real* SNICE, real* SNLIQ, real* sneqv) {
  int NEWNODE = 0;
  if (*ISNOW == 0 && QSNOW > K(0.0)) {
    *snowh = *snowh + snowhin * DT;
    *sneqv = *sneqv + QSNOW * DT;
  }
  if (*ISNOW == 0 && QSNOW > K(0.0) && *snowh >= K(0.025)) {
    *ISNOW = -1;
    NEWNODE = 1;
    DZSNSO[0] = *snowh;
    *snowh = K(0.0);
    STC[0] = rmin(K(273.16), SFCTMP);
    SNICE[0] = *sneqv;
    SNLIQ[0] = K(0.0);
  }
  if (*ISNOW < 0 && NEWNODE == 0 && QSNOW > K(0.0)) {
    SNICE[*ISNOW + 1] = SNICE[*ISNOW + 1] + QSNOW * DT;
    DZSNSO[*ISNOW + 1] = DZSNSO[*ISNOW + 1] + snowhin * DT;
  }
}

/* combo: func.f90:5536-5577 */
static void combo(real* DZ, real* WLIQ, real* WICE, real* T, real DZ2, real WLIQ2, real WICE2,
                  real T2) {
  real DZC = *DZ + DZ2;
  real WICEC = *WICE + WICE2;
  real WLIQC = *WLIQ + WLIQ2;
  real H = (CICE * *WICE + CWAT * *WLIQ) * (*T - TFRZ) + HFUS * *WLIQ;
  real H2 = (CICE * WICE2 + CWAT * WLIQ2) * (T2 - TFRZ) + HFUS * WLIQ2;
  real HC = H + H2;
  real TC;
  if (HC < K(0.0))
    TC = TFRZ + HC / (CICE * WICEC + CWAT * WLIQC);
  else if (HC <= HFUS * WLIQC)
    TC = TFRZ;
  else
    TC = TFRZ + (HC - HFUS * WLIQC) / (CICE * WICEC + CWAT * WLIQC);
  *DZ = DZC;
  *WICE = WICEC;
  *WLIQ = WLIQC;
  *T = TC;
}

/* combine: func.f90:5236-5413 (PONDING1/2 only assigned on some paths, H3) */
static void combine(int* ISNOW, real* soilwat, real* STC, real* SNICE, real* SNLIQ, real* DZSNSO,
                    real* soilice, real* snowh, real* sneqv, real* PONDING1, real* PONDING2) {
  const real DZMIN[3] = {K(0.025), K(0.025), K(0.1)};
  int ISNOW_OLD = *ISNOW;
  for (int J = ISNOW_OLD + 1; J <= 0; ++J) {
    if (SNICE[J] <= K(0.1)) {
      if (J != 0) {
        SNLIQ[J + 1] = SNLIQ[J + 1] + SNLIQ[J];
        SNICE[J + 1] = SNICE[J + 1] + SNICE[J];
      } else {
        if (ISNOW_OLD < -1) {
          SNLIQ[J - 1] = SNLIQ[J - 1] + SNLIQ[J];
          SNICE[J - 1] = SNICE[J - 1] + SNICE[J];
        } else {
          if (SNICE[J] >= K(0.0)) {
            *PONDING1 = SNLIQ[J];
            *sneqv = SNICE[J];
            *snowh = DZSNSO[J];
          } else {
            *PONDING1 = SNLIQ[J] + SNICE[J];
            if (*PONDING1 < K(0.0)) {
              soilice[1] = rmax(K(0.0), soilice[1] + *PONDING1 / (DZSNSO[1] * K(1000.0)));
              *PONDING1 = K(0.0);
            }
            *sneqv = K(0.0);
            *snowh = K(0.0);
          }
          SNLIQ[J] = K(0.0);
          SNICE[J] = K(0.0);
          DZSNSO[J] = K(0.0);
        }
      }
      if (J > *ISNOW + 1 && *ISNOW < -1) {
        for (int I = J; I >= *ISNOW + 2; --I) {
          STC[I] = STC[I - 1];
          SNLIQ[I] = SNLIQ[I - 1];
          SNICE[I] = SNICE[I - 1];
          DZSNSO[I] = DZSNSO[I - 1];
        }
      }
      *ISNOW = *ISNOW + 1;
    }
  }
  if (soilice[1] < K(0.0)) {
    soilwat[1] = soilwat[1] + soilice[1];
    soilice[1] = K(0.0);
  }
  if (*ISNOW == 0) return;
  *sneqv = K(0.0);
  *snowh = K(0.0);
  real ZWICE = K(0.0), ZWLIQ = K(0.0);
  for (int J = *ISNOW + 1; J <= 0; ++J) {
    *sneqv = *sneqv + SNICE[J] + SNLIQ[J];
    *snowh = *snowh + DZSNSO[J];
    ZWICE = ZWICE + SNICE[J];
    ZWLIQ = ZWLIQ + SNLIQ[J];
  }
  if (*snowh < K(0.025) && *ISNOW < 0) {
    *ISNOW = 0;
    *sneqv = ZWICE;
    *PONDING2 = ZWLIQ;
    if (*sneqv <= K(0.0)) *snowh = K(0.0);
  }
  if (*ISNOW < -1) {
    ISNOW_OLD = *ISNOW;
    int MSSI = 1;
    for (int I = ISNOW_OLD + 1; I <= 0; ++I) {
      if (DZSNSO[I] < DZMIN[MSSI - 1]) {
        int NEIBOR;
        if (I == *ISNOW + 1) {
          NEIBOR = I + 1;
        } else if (I == 0) {
          NEIBOR = I - 1;
        } else {
          NEIBOR = I + 1;
          if ((DZSNSO[I - 1] + DZSNSO[I]) < (DZSNSO[I + 1] + DZSNSO[I])) NEIBOR = I - 1;
        }
        int J, L;
        if (NEIBOR > I) {
          J = NEIBOR;
          L = I;
        } else {
          J = I;
          L = NEIBOR;
        }
        combo(&DZSNSO[J], &SNLIQ[J], &SNICE[J], &STC[J], DZSNSO[L], SNLIQ[L], SNICE[L], STC[L]);
        if (J - 1 > *ISNOW + 1) {
          for (int Kk = J - 1; Kk >= *ISNOW + 2; --Kk) {
            STC[Kk] = STC[Kk - 1];
            SNICE[Kk] = SNICE[Kk - 1];
            SNLIQ[Kk] = SNLIQ[Kk - 1];
            DZSNSO[Kk] = DZSNSO[Kk - 1];
          }
        }
        *ISNOW = *ISNOW + 1;
        if (*ISNOW >= -1) break;
      } else {
        MSSI = MSSI + 1;
      }
    }
  }
}

/* divide: func.f90:5416-5533 */
static void divide(int* ISNOW, real* STC, real* SNICE, real* SNLIQ, real* DZSNSO) {
  real DZ[4] = {0, 0, 0, 0}, SWICE[4] = {0, 0, 0, 0}, SWLIQ[4] = {0, 0, 0, 0},
       TSNO[4] = {0, 0, 0, 0}; /* 1-based */
  for (int J = 1; J <= NSNOW; ++J) {
    if (J <= abs(*ISNOW)) {
      DZ[J] = DZSNSO[J + *ISNOW];
      SWICE[J] = SNICE[J + *ISNOW];
      SWLIQ[J] = SNLIQ[J + *ISNOW];
      TSNO[J] = STC[J + *ISNOW];
    }
  }
  int MSNO = abs(*ISNOW);
  if (MSNO == 1) {
    if (DZ[1] > K(0.05)) {
      MSNO = 2;
      DZ[1] = DZ[1] / K(2.0);
      SWICE[1] = SWICE[1] / K(2.0);
      SWLIQ[1] = SWLIQ[1] / K(2.0);
      DZ[2] = DZ[1];
      SWICE[2] = SWICE[1];
      SWLIQ[2] = SWLIQ[1];
      TSNO[2] = TSNO[1];
    }
  }
  if (MSNO > 1) {
    if (DZ[1] > K(0.05)) {
      real DRR = DZ[1] - K(0.05);
      real PROPOR = DRR / DZ[1];
      real ZWICE = PROPOR * SWICE[1];
      real ZWLIQ = PROPOR * SWLIQ[1];
      PROPOR = K(0.05) / DZ[1];
      SWICE[1] = PROPOR * SWICE[1];
      SWLIQ[1] = PROPOR * SWLIQ[1];
      DZ[1] = K(0.05);
      combo(&DZ[2], &SWLIQ[2], &SWICE[2], &TSNO[2], DRR, ZWLIQ, ZWICE, TSNO[1]);
      if (MSNO <= 2 && DZ[2] > K(0.20)) {
        MSNO = 3;
        real DTDZ = (TSNO[1] - TSNO[2]) / ((DZ[1] + DZ[2]) / K(2.));
        DZ[2] = DZ[2] / K(2.0);
        SWICE[2] = SWICE[2] / K(2.0);
        SWLIQ[2] = SWLIQ[2] / K(2.0);
        DZ[3] = DZ[2];
        SWICE[3] = SWICE[2];
        SWLIQ[3] = SWLIQ[2];
        TSNO[3] = TSNO[2] - DTDZ * DZ[2] / K(2.0);
        if (TSNO[3] >= TFRZ)
          TSNO[3] = TSNO[2];
        else
          TSNO[2] = TSNO[2] + DTDZ * DZ[2] / K(2.0);
      }
    }
  }
  if (MSNO > 2) {
    if (DZ[2] > K(0.2)) {
      real DRR = DZ[2] - K(0.2);
      real PROPOR = DRR / DZ[2];
      real ZWICE = PROPOR * SWICE[2];
      real ZWLIQ = PROPOR * SWLIQ[2];
      PROPOR = K(0.2) / DZ[2];
      SWICE[2] = PROPOR * SWICE[2];
      SWLIQ[2] = PROPOR * SWLIQ[2];
      DZ[2] = K(0.2);
      combo(&DZ[3], &SWLIQ[3], &SWICE[3], &TSNO[3], DRR, ZWLIQ, ZWICE, TSNO[2]);
    }
  }
  *ISNOW = -MSNO;
  for (int J = *ISNOW + 1; J <= 0; ++J) {
    DZSNSO[J] = DZ[J - *ISNOW];
    SNICE[J] = SWICE[J - *ISNOW];
    SNLIQ[J] = SWLIQ[J - *ISNOW];
    STC[J] = TSNO[J - *ISNOW];
  }
}

/* compact: func.f90:5580-5677 */
static void compact(real DT, const real* STC, const real* SNICE, const real* SNLIQ,
                    const int* IMELT, const real* FICEOLD, int ISNOW, real* DZSNSO) {
  const real C2 = K(21.e-3), C3 = K(2.5e-6), C4 = K(0.04), C5 = K(2.0), DM = K(100.0),
             ETA0 = K(0.8e+6);
  real BURDEN = K(0.0);
  for (int J = ISNOW + 1; J <= 0; ++J) {
    real WX = SNICE[J] + SNLIQ[J];
    real FICE = SNICE[J] / WX;
    real VOID = K(1.) - (SNICE[J] / DENICE + SNLIQ[J] / DENWAT) / DZSNSO[J];
    if (VOID > K(0.001) && SNICE[J] > K(0.1)) {
      real BI = SNICE[J] / DZSNSO[J];
      real TD = rmax(K(0.0), TFRZ - STC[J]);
      real DEXPF = EXP(-C4 * TD);
      real DDZ1 = -C3 * DEXPF;
      if (BI > DM) DDZ1 = DDZ1 * EXP(K(-46.0E-3) * (BI - DM));
      if (SNLIQ[J] > K(0.01) * DZSNSO[J]) DDZ1 = DDZ1 * C5;
      real DDZ2 = -(BURDEN + K(0.5) * WX) * EXP(K(-0.08) * TD - C2 * BI) / ETA0;
      real DDZ3;
      if (IMELT[J] == 1) {
        DDZ3 = rmax(K(0.0), (FICEOLD[J] - FICE) / rmax(K(1.E-6), FICEOLD[J]));
        DDZ3 = -DDZ3 / DT;
      } else {
        DDZ3 = K(0.0);
      }
      real PDZDTC = (DDZ1 + DDZ2 + DDZ3) * DT;
      PDZDTC = rmax(K(-0.5), PDZDTC);
      DZSNSO[J] = DZSNSO[J] * (K(1.0) + PDZDTC);
    }
    BURDEN = BURDEN + WX;
  }
}

/* snowh2o: func.f90:5680-5819 */
static void snowh2o(const nmp_params* P, real DT, real QSNFRO, real QSNSUB, real QRAIN,
                    int* ISNOW, real* DZSNSO, real* snowh, real* sneqv, real* SNICE, real* SNLIQ,
                    real* soilwat, real* soilice, real* STC, real* QSNBOT, real* PONDING1,
                    real* PONDING2) {
  real VOL_LIQb[3] = {0, 0, 0}, VOL_ICEb[3] = {0, 0, 0}, eporeb[3] = {0, 0, 0};
  real *VOL_LIQ = VOL_LIQb + 2, *VOL_ICE = VOL_ICEb + 2, *epore = eporeb + 2;
  if (*sneqv == K(0.0)) {
    soilice[1] = soilice[1] + (QSNFRO - QSNSUB) * DT / (DZSNSO[1] * K(1000.0));
    if (soilice[1] < K(0.0)) {
      soilwat[1] = soilwat[1] + soilice[1];
      soilice[1] = K(0.0);
    }
  }
  if (*ISNOW == 0 && *sneqv > K(0.0)) {
    real TEMP = *sneqv;
    *sneqv = *sneqv - QSNSUB * DT + QSNFRO * DT;
    real PROPOR = *sneqv / TEMP;
    *snowh = rmax(K(0.0), PROPOR * *snowh);
    if (*sneqv < K(0.0)) {
      soilice[1] = soilice[1] + *sneqv / (DZSNSO[1] * K(1000.0));
      *sneqv = K(0.0);
      *snowh = K(0.0);
    }
    if (soilice[1] < K(0.0)) {
      soilwat[1] = soilwat[1] + soilice[1];
      soilice[1] = K(0.0);
    }
  }
  if (*snowh <= K(1.0E-8) || *sneqv <= K(1.0E-6)) {
    *snowh = K(0.0);
    *sneqv = K(0.0);
  }
  if (*ISNOW < 0) {
    real WGDIF = SNICE[*ISNOW + 1] - QSNSUB * DT + QSNFRO * DT;
    SNICE[*ISNOW + 1] = WGDIF;
    if (WGDIF < K(1.0E-6) && *ISNOW < 0)
      combine(ISNOW, soilwat, STC, SNICE, SNLIQ, DZSNSO, soilice, snowh, sneqv, PONDING1, PONDING2);
    if (*ISNOW < 0) {
      SNLIQ[*ISNOW + 1] = SNLIQ[*ISNOW + 1] + QRAIN * DT;
      SNLIQ[*ISNOW + 1] = rmax(K(0.0), SNLIQ[*ISNOW + 1]);
    }
  }
  for (int J = -NSNOW + 1; J <= 0; ++J) {
    if (J >= *ISNOW + 1) {
      VOL_ICE[J] = rmin(K(1.0), SNICE[J] / (DZSNSO[J] * DENICE));
      epore[J] = K(1.0) - VOL_ICE[J];
      VOL_LIQ[J] = rmin(epore[J], SNLIQ[J] / (DZSNSO[J] * DENWAT));
    }
  }
  real QIN = K(0.0), QOUT = K(0.0);
  for (int J = -NSNOW + 1; J <= 0; ++J) {
    if (J >= *ISNOW + 1) {
      SNLIQ[J] = SNLIQ[J] + QIN;
      if (J <= -1) {
        if (epore[J] < K(0.05) || epore[J + 1] < K(0.05)) {
          QOUT = K(0.0);
        } else {
          QOUT = rmax(K(0.0), (VOL_LIQ[J] - (real)P->ssi * epore[J]) * DZSNSO[J]);
          QOUT = rmin(QOUT, (K(1.0) - VOL_ICE[J + 1] - VOL_LIQ[J + 1]) * DZSNSO[J + 1]);
        }
      } else {
        QOUT = rmax(K(0.0), (VOL_LIQ[J] - (real)P->ssi * epore[J]) * DZSNSO[J]);
      }
      QOUT = QOUT * K(1000.0);
      SNLIQ[J] = SNLIQ[J] - QOUT;
      QIN = QOUT;
    }
  }
  *QSNBOT = QOUT / DT;
}

/* snowwater: func.f90:5049-5174 */
static void snowwater(ctx_t* X, real dt, const real* zsoil, const int* IMELT, real SFCTMP,
                      real snowhin, real QSNOW, real QSNFRO, real QSNSUB, real QRAIN,
                      const real* FICEOLD, int* ISNOW, real* snowh, real* sneqv, real* SNICE,
                      real* SNLIQ, real* soilwat, real* soilice, real* STC, real* ZSNSO,
                      real* DZSNSO, real* QSNBOT, real* SNOFLOW, real* PONDING1,
                      real* PONDING2) {
  *SNOFLOW = K(0.0);
  *PONDING1 = K(0.0);
  *PONDING2 = K(0.0);
  snowfall(dt, QSNOW, snowhin, SFCTMP, ISNOW, snowh, DZSNSO, STC, SNICE, SNLIQ, sneqv);
  if (*ISNOW < 0) compact(dt, STC, SNICE, SNLIQ, IMELT, FICEOLD, *ISNOW, DZSNSO);
  if (*ISNOW < 0)
    combine(ISNOW, soilwat, STC, SNICE, SNLIQ, DZSNSO, soilice, snowh, sneqv, PONDING1, PONDING2);
  if (*ISNOW < 0) divide(ISNOW, STC, SNICE, SNLIQ, DZSNSO);
  snowh2o(X->P, dt, QSNFRO, QSNSUB, QRAIN, ISNOW, DZSNSO, snowh, sneqv, SNICE, SNLIQ, soilwat,
          soilice, STC, QSNBOT, PONDING1, PONDING2);
  for (int iz = -NSNOW + 1; iz <= *ISNOW; ++iz) {
    SNICE[iz] = K(0.0);
    SNLIQ[iz] = K(0.0);
    STC[iz] = K(0.0);
    DZSNSO[iz] = K(0.0);
    ZSNSO[iz] = K(0.0);
  }
  if (*sneqv > K(2000.0)) {
    real BDSNOW = SNICE[0] / DZSNSO[0];
    *SNOFLOW = (*sneqv - K(2000.0));
    SNICE[0] = SNICE[0] - *SNOFLOW;
    DZSNSO[0] = DZSNSO[0] - *SNOFLOW / BDSNOW;
    *SNOFLOW = *SNOFLOW / dt;
  }
  if (*ISNOW < 0) {
    *sneqv = K(0.0);
    for (int IZ = *ISNOW + 1; IZ <= 0; ++IZ) *sneqv = *sneqv + SNICE[IZ] + SNLIQ[IZ];
  }
  for (int IZ = *ISNOW + 1; IZ <= 0; ++IZ) DZSNSO[IZ] = -DZSNSO[IZ];
  DZSNSO[1] = zsoil[1];
  for (int IZ = 2; IZ <= NSOIL; ++IZ) DZSNSO[IZ] = (zsoil[IZ] - zsoil[IZ - 1]);
  ZSNSO[*ISNOW + 1] = DZSNSO[*ISNOW + 1];
  for (int IZ = *ISNOW + 2; IZ <= NSOIL; ++IZ) ZSNSO[IZ] = ZSNSO[IZ - 1] + DZSNSO[IZ];
  for (int IZ = *ISNOW + 1; IZ <= NSOIL; ++IZ) DZSNSO[IZ] = -DZSNSO[IZ];
}

/* wdfcnd1: func.f90:4386-4417 */
static void wdfcnd1(const nmp_params* P, int sltyp, real* WDF, real* WCND, real SMC, real FCR) {
  real FACTR = rmax(K(0.01), SMC / SOILP(smcmax));
  real EXPON = SOILP(bexp) + K(2.0);
  *WDF = SOILP(dwsat) * POW(FACTR, EXPON);
  *WDF = *WDF * (K(1.0) - FCR);
  EXPON = K(2.0) * SOILP(bexp) + K(3.0);
  *WCND = SOILP(dksat) * POW(FACTR, EXPON);
  *WCND = *WCND * (K(1.0) - FCR);
}

/* wdfcnd2: func.f90:4420-4455 */
static void wdfcnd2(const nmp_params* P, int sltyp, real* WDF, real* WCND, real SMC,
                    real soilice) {
  real FACTR = rmax(K(0.01), SMC / SOILP(smcmax));
  real EXPON = SOILP(bexp) + K(2.0);
  *WDF = SOILP(dwsat) * POW(FACTR, EXPON);
  if (soilice > K(0.0)) {
    real VKWGT = K(1.0) / (K(1.0) + p3(K(500.0) * soilice));
    *WDF = VKWGT * *WDF + (K(1.0) - VKWGT) * SOILP(dwsat) * POW(K(0.2) / SOILP(smcmax), EXPON);
  }
  EXPON = K(2.0) * SOILP(bexp) + K(3.0);
  *WCND = SOILP(dksat) * POW(FACTR, EXPON);
}

/* zwteq (opt_run=2): func.f90:6051-6100 */
static void zwteq(const nmp_params* P, int sltyp, const real* ZSOIL, const real* DZSNSO,
                  const real* soilwat, real* ZWT) {
  const int NFINE = 100;
  real WD1 = K(0.0);
  for (int k = 1; k <= NSOIL; ++k) WD1 = WD1 + (SOILP(smcmax) - soilwat[k]) * DZSNSO[k];
  real DZFINE = K(3.0) * (-ZSOIL[NSOIL]) / (real)NFINE;
  *ZWT = K(-3.0) * ZSOIL[NSOIL] - K(0.001);
  real WD2 = K(0.0);
  for (int k = 1; k <= NFINE; ++k) {
    real ZFINE = (real)k * DZFINE;
    real TEMP = K(1.0) + (*ZWT - ZFINE) / SOILP(psisat);
    WD2 = WD2 + SOILP(smcmax) * (K(1.0) - POW(TEMP, K(-1.0) / SOILP(bexp))) * DZFINE;
    if (FABS(WD2 - WD1) <= K(0.01)) {
      *ZWT = ZFINE;
      break;
    }
  }
}

/* infil (opt_run=3): func.f90:6103-6196 */
static void infil(const nmp_params* P, int sltyp, real dt, const real* zsoil,
                  const real* soilwat, const real* soilice, real SICEMAX, real qinsrf,
                  real* qinfil, real* runsrf) {
  if (qinsrf > K(0.0)) {
    real DT1 = dt / K(86400.0);
    real SMCAV = SOILP(smcmax) - SOILP(smcwlt);
    real DMAX[NSOIL + 1];
    DMAX[1] = -zsoil[1] * SMCAV;
    real DICE = -zsoil[1] * soilice[1];
    DMAX[1] = DMAX[1] * (K(1.0) - (soilwat[1] + soilice[1] - SOILP(smcwlt)) / SMCAV);
    real DD = DMAX[1];
    for (int k = 2; k <= NSOIL; ++k) {
      DICE = DICE + (zsoil[k - 1] - zsoil[k]) * soilice[k];
      DMAX[k] = (zsoil[k - 1] - zsoil[k]) * SMCAV;
      DMAX[k] = DMAX[k] * (K(1.0) - (soilwat[k] + soilice[k] - SOILP(smcwlt)) / SMCAV);
      DD = DD + DMAX[k];
    }
    real VAL = (K(1.0) - EXP(-SOILP(kdt) * DT1));
    real DDT = DD * VAL;
    real PX = rmax(K(0.0), qinsrf * dt);
    real INFMAX = (PX * (DDT / (PX + DDT))) / dt;
    real FCR = K(1.0);
    if (DICE > K(1.0E-2)) {
      const int CVFRZ = 3;
      real ACRT = (real)CVFRZ * SOILP(frzx) / DICE;
      real SUM = K(1.0);
      int IALP1 = CVFRZ - 1;
      for (int J = 1; J <= IALP1; ++J) {
        int KK = 1;
        for (int JJ = J + 1; JJ <= IALP1; ++JJ) KK = KK * JJ;
        real ap = K(1.0);
        for (int e = 0; e < CVFRZ - J; ++e) ap = ap * ACRT;
        SUM = SUM + ap / (real)KK;
      }
      FCR = K(1.0) - EXP(-ACRT) * SUM;
    }
    INFMAX = INFMAX * FCR;
    real WDF, WCND;
    wdfcnd2(P, sltyp, &WDF, &WCND, soilwat[1], SICEMAX);
    INFMAX = rmax(INFMAX, WCND);
    INFMAX = rmin(INFMAX, PX);
    *runsrf = rmax(K(0.0), qinsrf - INFMAX);
    *qinfil = qinsrf - *runsrf;
  }
}

/* srt: func.f90:6199-6305 */
static void srt(ctx_t* X, int sltyp, const real* zsoil, int slptyp, real qinfil,
                const real* ETRANI, real QSEVA, const real* soilwat, const real* SMC,
                const real* FCR, real SICEMAX, real FCRMAX, real* RHSTT, real* AI, real* BI,
                real* CI, real* QDRAIN, real* WCND) {
  const nmp_params* P = X->P;
  real DDZ[NSOIL + 1], DENOM[NSOIL + 1], DSMDZ[NSOIL + 1], WFLUX[NSOIL + 1], WDF[NSOIL + 1],
      SMX[NSOIL + 1];
  if (X->O->opt_inf == 1) {
    for (int k = 1; k <= NSOIL; ++k) {
      wdfcnd1(P, sltyp, &WDF[k], &WCND[k], SMC[k], FCR[k]);
      SMX[k] = SMC[k];
    }
  }
  if (X->O->opt_inf == 2) {
    for (int k = 1; k <= NSOIL; ++k) {
      wdfcnd2(P, sltyp, &WDF[k], &WCND[k], soilwat[k], SICEMAX);
      SMX[k] = soilwat[k];
    }
  }
  const int orun = X->O->opt_run;
  for (int k = 1; k <= NSOIL; ++k) {
    if (k == 1) {
      DENOM[k] = -zsoil[k];
      real TEMP1 = -zsoil[k + 1];
      DDZ[k] = K(2.0) / TEMP1;
      DSMDZ[k] = K(2.0) * (SMX[k] - SMX[k + 1]) / TEMP1;
      WFLUX[k] = WDF[k] * DSMDZ[k] + WCND[k] - qinfil + ETRANI[k] + QSEVA;
    } else if (k < NSOIL) {
      DENOM[k] = (zsoil[k - 1] - zsoil[k]);
      real TEMP1 = (zsoil[k - 1] - zsoil[k + 1]);
      DDZ[k] = K(2.0) / TEMP1;
      DSMDZ[k] = K(2.0) * (SMX[k] - SMX[k + 1]) / TEMP1;
      WFLUX[k] = WDF[k] * DSMDZ[k] + WCND[k] - WDF[k - 1] * DSMDZ[k - 1] - WCND[k - 1] + ETRANI[k];
    } else {
      DENOM[k] = (zsoil[k - 1] - zsoil[k]);
      if (orun == 1 || orun == 2) *QDRAIN = K(0.0);
      if (orun == 3) *QDRAIN = (real)P->slope[slptyp - 1] * WCND[k];
      if (orun == 4) *QDRAIN = (K(1.0) - FCRMAX) * WCND[k];
      WFLUX[k] = -(WDF[k - 1] * DSMDZ[k - 1]) - WCND[k - 1] + ETRANI[k] + *QDRAIN;
    }
  }
  for (int k = 1; k <= NSOIL; ++k) {
    if (k == 1) {
      AI[k] = K(0.0);
      BI[k] = WDF[k] * DDZ[k] / DENOM[k];
      CI[k] = -BI[k];
    } else if (k < NSOIL) {
      AI[k] = -WDF[k - 1] * DDZ[k - 1] / DENOM[k];
      CI[k] = -WDF[k] * DDZ[k] / DENOM[k];
      BI[k] = -(AI[k] + CI[k]);
    } else {
      AI[k] = -WDF[k - 1] * DDZ[k - 1] / DENOM[k];
      CI[k] = K(0.0);
      BI[k] = -(AI[k] + CI[k]);
    }
    RHSTT[k] = WFLUX[k] / (-DENOM[k]);
  }
}

/* sstep: func.f90:6308-6383 */
static void sstep(const nmp_params* P, int sltyp, real dt, const real* dzsnso, const real* soilice,
                  real* soilwat, real* SMC, real* AI, real* BI, real* CI, real* RHSTT,
                  real* WPLUS) {
  real RHSTTIN[NSOIL + 1], CIIN[NSOIL + 1];
  *WPLUS = K(0.0);
  for (int k = 1; k <= NSOIL; ++k) {
    RHSTT[k] = RHSTT[k] * dt;
    AI[k] = AI[k] * dt;
    BI[k] = K(1.0) + BI[k] * dt;
    CI[k] = CI[k] * dt;
  }
  for (int k = 1; k <= NSOIL; ++k) {
    RHSTTIN[k] = RHSTT[k];
    CIIN[k] = CI[k];
  }
  rosr12(CI, AI, BI, CIIN, RHSTTIN, RHSTT, 1, NSOIL);
  for (int k = 1; k <= NSOIL; ++k) soilwat[k] = soilwat[k] + CI[k];
  real epore;
  for (int k = NSOIL; k >= 2; --k) {
    epore = rmax(K(1.0E-4), SOILP(smcmax) - soilice[k]);
    *WPLUS = rmax(soilwat[k] - epore, K(0.0)) * dzsnso[k];
    soilwat[k] = rmin(epore, soilwat[k]);
    soilwat[k - 1] = soilwat[k - 1] + *WPLUS / dzsnso[k - 1];
  }
  epore = rmax(K(1.0E-4), SOILP(smcmax) - soilice[1]);
  *WPLUS = rmax(soilwat[1] - epore, K(0.0)) * dzsnso[1];
  soilwat[1] = rmin(epore, soilwat[1]);
  for (int k = 1; k <= NSOIL; ++k) SMC[k] = soilwat[k] + soilice[k];
}

/* soilh2o: func.f90:5822-6048 */
static void soilh2o(ctx_t* X, int sltyp, int lutyp, real dt, const real* zsoil,
                    const real* dzsnso, int slptyp, real qinsrf, real QSEVA, const real* ETRANI,
                    const real* soilice, real* soilwat, real* SMC, real* ZWT, real* runsrf,
                    real* QDRAIN, real* runsub, real* WCND, real* FCRMAX) {
  const nmp_params* P = X->P;
  const int orun = X->O->opt_run;
  const real A = K(4.0);
  real RHSTT[NSOIL + 1], AI[NSOIL + 1], BI[NSOIL + 1], CI[NSOIL + 1], FCR[NSOIL + 1],
      MLIQ[NSOIL + 1];
  *runsrf = K(0.0);
  real qinfil = K(0.0);
  real RSAT = K(0.0);
  for (int iz = 1; iz <= NSOIL; ++iz) {
    real epore = rmax(K(1.0E-4), (SOILP(smcmax) - soilice[iz]));
    RSAT = RSAT + rmax(K(0.0), soilwat[iz] - epore) * dzsnso[iz];
    soilwat[iz] = rmin(epore, soilwat[iz]);
  }
  for (int iz = 1; iz <= NSOIL; ++iz) {
    real FICE = rmin(K(1.0), soilice[iz] / SOILP(smcmax));
    FCR[iz] = rmax(K(0.0), EXP(-A * (K(1.0) - FICE)) - EXP(-A)) / (K(1.0) - EXP(-A));
  }
  real SICEMAX = K(0.0);
  *FCRMAX = K(0.0);
  real SH2OMIN = SOILP(smcmax);
  for (int iz = 1; iz <= NSOIL; ++iz) {
    if (soilice[iz] > SICEMAX) SICEMAX = soilice[iz];
    if (FCR[iz] > *FCRMAX) *FCRMAX = FCR[iz];
    if (soilwat[iz] < SH2OMIN) SH2OMIN = soilwat[iz];
  }
  real FFF, FSAT;
  if (orun == 2) {
    FFF = K(2.0);
    real RSBMX = K(4.0);
    zwteq(P, sltyp, zsoil, dzsnso, soilwat, ZWT);
    *runsub = (K(1.0) - *FCRMAX) * RSBMX * EXP(-(real)P->timean) * EXP(-FFF * *ZWT);
  }
  if (lutyp == P->isurban) FCR[1] = K(0.95);
  if (orun == 1) {
    FFF = K(6.0);
    FSAT = (real)P->fsatmax * EXP(K(-0.5) * FFF * (*ZWT - K(2.0)));
    if (qinsrf > K(0.0)) {
      *runsrf = qinsrf * ((K(1.0) - FCR[1]) * FSAT + FCR[1]);
      qinfil = qinsrf - *runsrf;
    }
  }
  if (orun == 2) {
    FFF = K(2.0);
    FSAT = (real)P->fsatmax * EXP(K(-0.5) * FFF * *ZWT);
    if (qinsrf > K(0.0)) {
      *runsrf = qinsrf * ((K(1.0) - FCR[1]) * FSAT + FCR[1]);
      qinfil = qinsrf - *runsrf;
    }
  }
  if (orun == 3) infil(P, sltyp, dt, zsoil, soilwat, soilice, SICEMAX, qinsrf, &qinfil, runsrf);
  if (orun == 4) {
    real SMCTOT = K(0.0), DZTOT = K(0.0);
    for (int iz = 1; iz <= NSOIL; ++iz) {
      DZTOT = DZTOT + dzsnso[iz];
      SMCTOT = SMCTOT + SMC[iz] * dzsnso[iz];
      if (DZTOT >= K(2.0)) break;
    }
    SMCTOT = SMCTOT / DZTOT;
    FSAT = POW(rmax(K(0.01), SMCTOT / SOILP(smcmax)), K(4.0));
    if (qinsrf > K(0.0)) {
      *runsrf = qinsrf * ((K(1.0) - FCR[1]) * FSAT + FCR[1]);
      qinfil = qinsrf - *runsrf;
    }
  }
  int niter = 1;
  if (X->O->opt_inf == 1) {
    niter = 3;
    if (qinfil * dt > dzsnso[1] * SOILP(smcmax)) niter = niter * 2;
  }
  real dtfine = dt / (real)niter;
  real QDRAIN_SAVE = K(0.0);
  for (int iter = 1; iter <= niter; ++iter) { ITER_STAT(3);
    real WPLUS;
    srt(X, sltyp, zsoil, slptyp, qinfil, ETRANI, QSEVA, soilwat, SMC, FCR, SICEMAX, *FCRMAX,
        RHSTT, AI, BI, CI, QDRAIN, WCND);
    sstep(P, sltyp, dtfine, dzsnso, soilice, soilwat, SMC, AI, BI, CI, RHSTT, &WPLUS);
    RSAT = RSAT + WPLUS;
    QDRAIN_SAVE = QDRAIN_SAVE + *QDRAIN;
  }
  *QDRAIN = QDRAIN_SAVE / (real)niter;
  *runsrf = *runsrf * K(1000.0) + RSAT * K(1000.0) / dt;
  *QDRAIN = *QDRAIN * K(1000.0);
  if (orun == 2) {
    real WTSUB = K(0.0);
    for (int iz = 1; iz <= NSOIL; ++iz) WTSUB = WTSUB + WCND[iz] * dzsnso[iz];
    for (int iz = 1; iz <= NSOIL; ++iz) {
      real MH2O = *runsub * dt * (WCND[iz] * dzsnso[iz]) / WTSUB;
      soilwat[iz] = soilwat[iz] - MH2O / (dzsnso[iz] * K(1000.0));
    }
  }
  if (orun != 1) {
    for (int iz = 1; iz <= NSOIL; ++iz) MLIQ[iz] = soilwat[iz] * dzsnso[iz] * K(1000.0);
    real WATMIN = K(0.01), XS;
    for (int iz = 1; iz <= NSOIL - 1; ++iz) {
      XS = (MLIQ[iz] < K(0.0)) ? WATMIN - MLIQ[iz] : K(0.0);
      MLIQ[iz] = MLIQ[iz] + XS;
      MLIQ[iz + 1] = MLIQ[iz + 1] - XS;
    }
    XS = (MLIQ[NSOIL] < WATMIN) ? WATMIN - MLIQ[NSOIL] : K(0.0);
    MLIQ[NSOIL] = MLIQ[NSOIL] + XS;
    *runsub = *runsub - XS / dt;
    for (int iz = 1; iz <= NSOIL; ++iz) soilwat[iz] = MLIQ[iz] / (dzsnso[iz] * K(1000.0));
  }
}

/* groundwater: func.f90:6458-6639 (S_NODE is real(8) in the reference) */
static void groundwater(const nmp_params* P, int sltyp, real DT, const real* ZSOIL,
                        const real* soilice, const real* WCND, real FCRMAX, real* soilwat,
                        real* ZWT, real* WA, real* WT, real* QIN, real* QDIS) {
  const real ROUS = K(0.2), CMIC = K(0.20);
  real DZMM[NSOIL + 1], ZNODE[NSOIL + 1], MLIQ[NSOIL + 1], epore[NSOIL + 1], HK[NSOIL + 1],
      SMC[NSOIL + 1];
  *QDIS = K(0.0);
  *QIN = K(0.0);
  DZMM[1] = -ZSOIL[1] * K(1.0E3);
  for (int iz = 2; iz <= NSOIL; ++iz) DZMM[iz] = K(1.0E3) * (ZSOIL[iz - 1] - ZSOIL[iz]);
  ZNODE[1] = -ZSOIL[1] / K(2.0);
  for (int iz = 2; iz <= NSOIL; ++iz)
    ZNODE[iz] = -ZSOIL[iz - 1] + K(0.5) * (ZSOIL[iz - 1] - ZSOIL[iz]);
  for (int iz = 1; iz <= NSOIL; ++iz) {
    SMC[iz] = soilwat[iz] + soilice[iz];
    MLIQ[iz] = soilwat[iz] * DZMM[iz];
    epore[iz] = rmax(K(0.01), SOILP(smcmax) - soilice[iz]);
    HK[iz] = K(1.0E3) * WCND[iz];
  }
  int IWT = NSOIL;
  for (int iz = 2; iz <= NSOIL; ++iz) {
    if (*ZWT <= -ZSOIL[iz]) {
      IWT = iz - 1;
      break;
    }
  }
  const real FFF = K(6.0), RSBMX = K(5.0);
  *QDIS = (K(1.0) - FCRMAX) * RSBMX * EXP(-(real)P->timean) * EXP(-FFF * (*ZWT - K(2.0)));
  double S_NODE = (double)rmin(K(1.0), SMC[IWT] / SOILP(smcmax));
  S_NODE = fmax(S_NODE, (double)0.01f);
  real SMPFZ = (real)(-((double)(SOILP(psisat) * K(1000.0)) * pow(S_NODE, (double)(-SOILP(bexp)))));
  SMPFZ = rmax(K(-120000.0), CMIC * SMPFZ);
  real KA = HK[IWT];
  real WH_ZWT = -*ZWT * K(1.0E3);
  real WH = SMPFZ - ZNODE[IWT] * K(1.0E3);
  *QIN = -KA * (WH_ZWT - WH) / ((*ZWT - ZNODE[IWT]) * K(1.0E3));
  *QIN = rmax(K(-10.0) / DT, rmin(K(10.0) / DT, *QIN));
  *WT = *WT + (*QIN - *QDIS) * DT;
  if (IWT == NSOIL) {
    *WA = *WA + (*QIN - *QDIS) * DT;
    *WT = *WA;
    *ZWT = (-ZSOIL[NSOIL] + K(25.0)) - *WA / K(1000.0) / ROUS;
    MLIQ[NSOIL] = MLIQ[NSOIL] - *QIN * DT;
    MLIQ[NSOIL] = MLIQ[NSOIL] + rmax(K(0.0), *WA - K(5000.0));
    *WA = rmin(*WA, K(5000.0));
  } else {
    if (IWT == NSOIL - 1) {
      *ZWT = -ZSOIL[NSOIL] - (*WT - ROUS * K(1000.0) * K(25.0)) / (epore[NSOIL]) / K(1000.0);
    } else {
      real WS = K(0.0);
      for (int iz = IWT + 2; iz <= NSOIL; ++iz) WS = WS + epore[iz] * DZMM[iz];
      *ZWT = -ZSOIL[IWT + 1] - (*WT - ROUS * K(1000.0) * K(25.0) - WS) / (epore[IWT + 1]) / K(1000.0);
    }
    real WTSUB = K(0.0);
    for (int iz = 1; iz <= NSOIL; ++iz) WTSUB = WTSUB + HK[iz] * DZMM[iz];
    for (int iz = 1; iz <= NSOIL; ++iz) MLIQ[iz] = MLIQ[iz] - *QDIS * DT * HK[iz] * DZMM[iz] / WTSUB;
  }
  *ZWT = rmax(K(1.5), *ZWT);
  real WATMIN = K(0.01), XS;
  for (int iz = 1; iz <= NSOIL - 1; ++iz) {
    XS = (MLIQ[iz] < K(0.0)) ? WATMIN - MLIQ[iz] : K(0.0);
    MLIQ[iz] = MLIQ[iz] + XS;
    MLIQ[iz + 1] = MLIQ[iz + 1] - XS;
  }
  XS = (MLIQ[NSOIL] < WATMIN) ? WATMIN - MLIQ[NSOIL] : K(0.0);
  MLIQ[NSOIL] = MLIQ[NSOIL] + XS;
  *WA = *WA - XS;
  *WT = *WT - XS;
  for (int iz = 1; iz <= NSOIL; ++iz) soilwat[iz] = MLIQ[iz] / DZMM[iz];
}

typedef struct {
  real ECAN, ETRAN, runsrf, runsub, QSNBOT, PONDING1, PONDING2, FPICE;
} waterout_t;

/* water: func.f90:4601-4804 */
static void water(ctx_t* X, int slptyp, int sltyp, int lutyp, real dt, const int* IMELT, real UU,
                  real VV, real FCEV, real FCTR, real QPRECC, real QPRECL, real elai, real esai,
                  real SFCTMP, real QVAP, real QDEW, const real* ZSOIL, const real* BTRANI,
                  const real* FICEOLD, real PONDING, real TG, int IST, real fveg,
                  int FROZEN_CANOPY, int FROZEN_GROUND, int* ISNOW, real* CANLIQ, real* CANICE,
                  real* TV, real* snowh, real* sneqv, real* SNICE, real* SNLIQ, real* STC,
                  real* ZSNSO, real* soilwat, real* SMC, real* soilice, real* ZWT, real* WA,
                  real* WT, real* DZSNSO, real* WSLAKE, real* FWET, real* QSNOW, waterout_t* o) {
  const nmp_params* P = X->P;
  real ETRANI[NSOIL + 1] = {0, 0, 0, 0, 0}, WCND[NSOIL + 1] = {0, 0, 0, 0, 0};
  real SNOFLOW = K(0.0), QIN = K(0.0), QDIS = K(0.0), QDRAIN = K(0.0), FCRMAX = K(0.0);
  o->runsub = K(0.0);
  real qinsrf = K(0.0), CMC, QRAIN, snowhin;
  canwater(X, lutyp, dt, SFCTMP, UU, VV, FCEV, FCTR, QPRECC, QPRECL, elai, esai, IST, TG, fveg,
           FROZEN_CANOPY, CANLIQ, CANICE, TV, &CMC, &o->ECAN, &o->ETRAN, &QRAIN, QSNOW, &snowhin,
           FWET, &o->FPICE);
  real QSNSUB = K(0.0);
  if (*sneqv > K(0.0)) QSNSUB = rmin(QVAP, *sneqv / dt);
  real QSEVA = QVAP - QSNSUB;
  real QSNFRO = K(0.0);
  if (*sneqv > K(0.0)) QSNFRO = QDEW;
  real QSDEW = QDEW - QSNFRO;
  snowwater(X, dt, ZSOIL, IMELT, SFCTMP, snowhin, *QSNOW, QSNFRO, QSNSUB, QRAIN, FICEOLD, ISNOW,
            snowh, sneqv, SNICE, SNLIQ, soilwat, soilice, STC, ZSNSO, DZSNSO, &o->QSNBOT,
            &SNOFLOW, &o->PONDING1, &o->PONDING2);
  if (FROZEN_GROUND) {
    soilice[1] = soilice[1] + (QSDEW - QSEVA) * dt / (DZSNSO[1] * K(1000.0));
    QSDEW = K(0.0);
    QSEVA = K(0.0);
    if (soilice[1] < K(0.0)) {
      soilwat[1] = soilwat[1] + soilice[1];
      soilice[1] = K(0.0);
    }
  }
  qinsrf = (PONDING + o->PONDING1 + o->PONDING2) / dt * K(0.001);
  if (*ISNOW == 0)
    qinsrf = qinsrf + (o->QSNBOT + QSDEW + QRAIN) * K(0.001);
  else
    qinsrf = qinsrf + (o->QSNBOT + QSDEW) * K(0.001);
  QSEVA = QSEVA * K(0.001);
  for (int iz = 1; iz <= P->nroot[lutyp - 1]; ++iz) ETRANI[iz] = o->ETRAN * BTRANI[iz] * K(0.001);
  if (IST == 2) {
    o->runsrf = K(0.);
    if (*WSLAKE >= K(5000.)) o->runsrf = qinsrf * K(1000.0);
    *WSLAKE = *WSLAKE + (qinsrf - QSEVA) * K(1000.0) * dt - o->runsrf * dt;
  } else {
    soilh2o(X, sltyp, lutyp, dt, ZSOIL, DZSNSO, slptyp, qinsrf, QSEVA, ETRANI, soilice, soilwat,
            SMC, ZWT, &o->runsrf, &QDRAIN, &o->runsub, WCND, &FCRMAX);
    if (X->O->opt_run == 1) {
      groundwater(P, sltyp, dt, ZSOIL, soilice, WCND, FCRMAX, soilwat, ZWT, WA, WT, &QIN, &QDIS);
      o->runsub = QDIS;
    }
    if (X->O->opt_run == 3 || X->O->opt_run == 4) o->runsub = o->runsub + QDRAIN;
    for (int iz = 1; iz <= NSOIL; ++iz) SMC[iz] = soilwat[iz] + soilice[iz];
  }
  o->runsub = o->runsub + SNOFLOW;
}

/* co2flux: func.f90:6754-7025 (called through carbon :6642-6751) */
static void carbon(const nmp_params* P, int lutyp, real DT, const real* ZSOIL, const real* DZSNSO,
                   const real* STC, const real* SMC, real TV, real PSN, real FOLN, real SMCMAX,
                   real BTRAN, real IGS, real* LFMASS, real* RTMASS, real* STMASS, real* WOOD,
                   real* STBLCP, real* FASTCP, real* GPP, real* NPP, real* NEE, real* XLAI,
                   real* XSAI) {
  if (lutyp == P->iswater || lutyp == P->isbarren || lutyp == P->isice || lutyp == P->isurban) {
    *XLAI = *XSAI = *GPP = *NPP = *NEE = K(0.0);
    *LFMASS = *RTMASS = *STMASS = *WOOD = *STBLCP = *FASTCP = K(0.0);
    return;
  }
  real LAPM = VEGP(sla) / K(1000.0);
  real WSTRES = K(1.0) - BTRAN;
  real WROOT = K(0.0);
  int nroot = P->nroot[lutyp - 1];
  for (int j = 1; j <= nroot; ++j) WROOT = WROOT + SMC[j] / SMCMAX * DZSNSO[j] / (-ZSOIL[nroot]);
  /* co2flux */
  const real RTOVRC = K(2.0E-8), RSWOODC = K(3.0E-10), BF = K(0.90), WSTRC = K(100.0),
             LAIMIN = K(0.05), XSAMIN = K(0.01);
  real SAPM = K(3.0) * K(0.001);
  real LFMSMN = LAIMIN / LAPM;
  real STMSMN = XSAMIN / SAPM;
  real RF = (IGS == K(0.0)) ? K(0.5) : K(1.0);
  real FNF = rmin(FOLN / rmax(K(1.0E-06), VEGP(folnmx)), K(1.0));
  real TF = POW(VEGP(arm), (TV - K(298.16)) / K(10.0));
  real RESP = VEGP(rmf25) * TF * FNF * *XLAI * RF * (K(1.0) - WSTRES);
  real RSLEAF = rmin(*LFMASS / DT, RESP * K(12.0E-6));
  real RSROOT = VEGP(rmr25) * (*RTMASS * K(1.0E-3)) * TF * RF * K(12.0E-6);
  real RSSTEM = VEGP(rms25) * (*STMASS * K(1.0E-3)) * TF * RF * K(12.0E-6);
  real RSWOOD = RSWOODC * EXP(K(0.08) * (TV - K(298.16))) * *WOOD * VEGP(wdpool);
  real CARBFX = PSN * K(12.0E-6);
  real LEAFPT = EXP(K(0.01) * (K(1.0) - EXP(K(0.75) * *XLAI)) * *XLAI);
  if (lutyp == P->isegblf) LEAFPT = EXP(K(0.01) * (K(1.0) - EXP(K(0.50) * *XLAI)) * *XLAI);
  real NONLEF = K(1.0) - LEAFPT;
  real STEMPT = *XLAI / K(10.0);
  LEAFPT = LEAFPT - STEMPT;
  real WOODF;
  if (*WOOD > K(0.0))
    WOODF = (K(1.0) - EXP(-BF * (VEGP(wrrat) * *RTMASS / *WOOD)) / BF) * VEGP(wdpool);
  else
    WOODF = K(0.0);
  real ROOTPT = NONLEF * (K(1.0) - WOODF);
  real WOODPT = NONLEF * WOODF;
  real LFTOVR = VEGP(ltovrc) * K(1.0E-6) * *LFMASS;
  real STTOVR = VEGP(ltovrc) * K(1.0E-6) * *STMASS;
  real RTTOVR = RTOVRC * *RTMASS;
  real WDTOVR = K(9.5E-10) * *WOOD;
  real SC = EXP(K(-0.3) * rmax(K(0.0), TV - VEGP(tdlef))) * (*LFMASS / K(120.0));
  real SD = EXP((WSTRES - K(1.0)) * WSTRC);
  real DIELF = *LFMASS * K(1.0E-6) * (VEGP(dilefw) * SD + VEGP(dilefc) * SC);
  real DIEST = *STMASS * K(1.0E-6) * (VEGP(dilefw) * SD + VEGP(dilefc) * SC);
  real GRLEAF = rmax(K(0.0), VEGP(fragr) * (LEAFPT * CARBFX - RSLEAF));
  real GRSTEM = rmax(K(0.0), VEGP(fragr) * (STEMPT * CARBFX - RSSTEM));
  real GRROOT = rmax(K(0.0), VEGP(fragr) * (ROOTPT * CARBFX - RSROOT));
  real GRWOOD = rmax(K(0.0), VEGP(fragr) * (WOODPT * CARBFX - RSWOOD));
  real ADDNPPLF = rmax(K(0.), LEAFPT * CARBFX - GRLEAF - RSLEAF);
  real ADDNPPST = rmax(K(0.), STEMPT * CARBFX - GRSTEM - RSSTEM);
  if (TV < VEGP(tmin)) ADDNPPLF = K(0.0);
  if (TV < VEGP(tmin)) ADDNPPST = K(0.0);
  real LFDEL = (*LFMASS - LFMSMN) / DT;
  real STDEL = (*STMASS - STMSMN) / DT;
  DIELF = rmin(DIELF, LFDEL + ADDNPPLF - LFTOVR);
  DIEST = rmin(DIEST, STDEL + ADDNPPST - STTOVR);
  real NPPL = rmax(ADDNPPLF, -LFDEL);
  real NPPS = rmax(ADDNPPST, -STDEL);
  real NPPR = ROOTPT * CARBFX - RSROOT - GRROOT;
  real NPPW = WOODPT * CARBFX - RSWOOD - GRWOOD;
  *LFMASS = *LFMASS + (NPPL - LFTOVR - DIELF) * DT;
  *STMASS = *STMASS + (NPPS - STTOVR - DIEST) * DT;
  *RTMASS = *RTMASS + (NPPR - RTTOVR) * DT;
  if (*RTMASS < K(0.0)) {
    RTTOVR = NPPR;
    *RTMASS = K(0.0);
  }
  *WOOD = (*WOOD + (NPPW - WDTOVR) * DT) * VEGP(wdpool);
  *FASTCP = *FASTCP + (RTTOVR + LFTOVR + STTOVR + WDTOVR + DIELF) * DT;
  real FST = EXP2((STC[1] - K(283.16)) / K(10.0));
  real FSW = WROOT / (K(0.20) + WROOT) * K(0.23) / (K(0.23) + WROOT);
  real RSSOIL = FSW * FST * VEGP(mrp) * rmax(K(0.0), *FASTCP * K(1.0E-3)) * K(12.0E-6);
  real STABLC = K(0.1) * RSSOIL;
  *FASTCP = *FASTCP - (RSSOIL + STABLC) * DT;
  *STBLCP = *STBLCP + STABLC * DT;
  *GPP = CARBFX;
  *NPP = NPPL + NPPW + NPPR;
  real AUTORS = RSROOT + RSWOOD + RSLEAF + GRLEAF + GRROOT + GRWOOD;
  real HETERS = RSSOIL;
  *NEE = (AUTORS + HETERS - *GPP) * K(44.0) / K(12.0);
  *XLAI = rmax(*LFMASS * LAPM, LAIMIN);
  *XSAI = rmax(*STMASS * SAPM, XSAMIN);
}

/* ------------------------------------------------------------------------ */
/* noahmp_sflx: func.f90:66-476, plus energy (735-1338) and error (633-732) */
static void sflx_column(ctx_t* X, real DT, int YEARLEN, real JULIAN, const real zsoil4[4],
                        real* s, int32_t* isnow_io, const real* sf, const int32_t* si,
                        const real* fc, real* d) {
  const nmp_params* P = X->P;
  const nmp_options* O = X->O;
  /* unpack (layout: include/noahmp_engine.h) */
  real STCb[7], ZSNSOb[7], DZSNSOb[7], SNICEb[3], SNLIQb[3], FICEOLDb[3];
  real *STC = STCb + 2, *ZSNSO = ZSNSOb + 2, *DZSNSO = DZSNSOb + 2, *SNICE = SNICEb + 2,
       *SNLIQ = SNLIQb + 2, *FICEOLD = FICEOLDb + 2;
  real soilwat[NSOIL + 1], SMC[NSOIL + 1], ZSOIL[NSOIL + 1], soilice[NSOIL + 1],
      BTRANI[NSOIL + 1];
  for (int k = 0; k < 7; ++k) {
    STCb[k] = s[NMP_S_STC + k];
    ZSNSOb[k] = s[NMP_S_ZSNSO + k];
    DZSNSOb[k] = K(0.0);
  }
  for (int k = 0; k < 3; ++k) {
    SNICEb[k] = s[NMP_S_SNICE + k];
    SNLIQb[k] = s[NMP_S_SNLIQ + k];
  }
  for (int k = 1; k <= NSOIL; ++k) {
    soilwat[k] = s[NMP_S_SH2O + k - 1];
    SMC[k] = s[NMP_S_SMC + k - 1];
    ZSOIL[k] = zsoil4[k - 1];
    soilice[k] = K(0.0);
    BTRANI[k] = K(0.0);
  }
  real TV = s[NMP_S_TV], TG = s[NMP_S_TG], TAH = s[NMP_S_TAH], EAH = s[NMP_S_EAH];
  real FWET = s[NMP_S_FWET], CANLIQ = s[NMP_S_CANLIQ], CANICE = s[NMP_S_CANICE];
  real QSFC = s[NMP_S_QSFC], snowh = s[NMP_S_SNOWH], sneqv = s[NMP_S_SNEQV];
  real SNEQVO = s[NMP_S_SNEQVO], ALBOLD = s[NMP_S_ALBOLD], TAUSS = s[NMP_S_TAUSS];
  real QSNOW = s[NMP_S_QSNOW], ZWT = s[NMP_S_ZWT], WA = s[NMP_S_WA], WT = s[NMP_S_WT];
  real WSLAKE = s[NMP_S_WSLAKE], LAI = s[NMP_S_LAI], SAI = s[NMP_S_SAI];
  real LFMASS = s[NMP_S_LFMASS], RTMASS = s[NMP_S_RTMASS], STMASS = s[NMP_S_STMASS];
  real WOOD = s[NMP_S_WOOD], STBLCP = s[NMP_S_STBLCP], FASTCP = s[NMP_S_FASTCP];
  real CM = s[NMP_S_CM], CH = s[NMP_S_CH];
  int ISNOW = *isnow_io;
  real LAT = sf[NMP_F_LAT], ZREF = sf[NMP_F_ZLVL], SHDFAC = sf[NMP_F_SHDFAC];
  real SHDMAX = sf[NMP_F_SHDMAX], TBOT = sf[NMP_F_TBOT], FOLN = sf[NMP_F_FOLN];
  int lutyp = si[NMP_I_VEGTYP], sltyp = si[NMP_I_SOILTYP], slptyp = si[NMP_I_SLOPETYP];
  int ISC = si[NMP_I_SOILCOLOR], IST = si[NMP_I_IST], ICE = si[NMP_I_ICE];
  real SFCTMP = fc[NMP_A_SFCTMP], SFCPRS = fc[NMP_A_SFCPRS], PSFC = fc[NMP_A_PSFC];
  real UU = fc[NMP_A_UU], VV = fc[NMP_A_VV], Q2 = fc[NMP_A_Q2], SOLDN = fc[NMP_A_SOLDN];
  real LWDN = fc[NMP_A_LWDN], PRCP = fc[NMP_A_PRCP], COSZ = fc[NMP_A_COSZ];
  real CO2AIR = fc[NMP_A_CO2AIR], O2AIR = fc[NMP_A_O2AIR];
  /* offline-driver FICEOLD: ice fraction of the active snow layers at step start */
  for (int iz = -2; iz <= 0; ++iz) FICEOLD[iz] = K(0.0);
  for (int iz = ISNOW + 1; iz <= 0; ++iz) FICEOLD[iz] = SNICE[iz] / (SNICE[iz] + SNLIQ[iz]);

  real NEE = K(0.0), NPP = K(0.0), GPP = K(0.0);
  real THAIR, QAIR, EAIR, RHOAIR, QPRECC, QPRECL, SOLAD[2], SOLAI[2], SWDOWN;
  atm(SFCPRS, SFCTMP, Q2, PRCP, SOLDN, COSZ, &THAIR, &QAIR, &EAIR, &RHOAIR, &QPRECC, &QPRECL,
      SOLAD, SOLAI, &SWDOWN);
  for (int IZ = ISNOW + 1; IZ <= NSOIL; ++IZ) {
    if (IZ == ISNOW + 1)
      DZSNSO[IZ] = -ZSNSO[IZ];
    else
      DZSNSO[IZ] = ZSNSO[IZ - 1] - ZSNSO[IZ];
  }
  const int nroot = P->nroot[lutyp - 1];
  real TROOT = K(0.0);
  for (int IZ = 1; IZ <= nroot; ++IZ) TROOT = TROOT + STC[IZ] * DZSNSO[IZ] / (-ZSOIL[nroot]);
  real BEG_WB = K(0.0);
  if (IST == 1) {
    BEG_WB = CANLIQ + CANICE + sneqv + WA;
    for (int IZ = 1; IZ <= NSOIL; ++IZ) BEG_WB = BEG_WB + SMC[IZ] * DZSNSO[IZ] * K(1000.0);
  }
  real HTOP, elai, esai, IGS;
  phenology(X, lutyp, snowh, TV, LAT, YEARLEN, JULIAN, &LAI, &SAI, &HTOP, &elai, &esai, &IGS);
  real fveg = K(0.0);
  if (O->opt_veg == 1) {
    fveg = SHDFAC;
    if (fveg <= K(0.01)) fveg = K(0.01);
  } else if (O->opt_veg == 2 || O->opt_veg == 3) {
    fveg = K(1.0) - EXP(K(-0.52) * (LAI + SAI));
    if (fveg <= K(0.01)) fveg = K(0.01);
  } else if (O->opt_veg == 4 || O->opt_veg == 5) {
    fveg = SHDMAX;
    if (fveg <= K(0.01)) fveg = K(0.01);
  } else {
    X->status |= NMP_ST_OPTVEG;
  }
  if (lutyp == P->isurban || lutyp == P->isbarren) fveg = K(0.0);
  if (elai + esai == K(0.0)) fveg = K(0.0);

  /* ===== energy: func.f90:735-1338 ===== */
  const real Z0 = K(0.01);
  real IRC = 0, SHC = 0, IRG = 0, SHG = 0, EVG = 0, EVC = 0, TR = 0, GHV = 0, PSNSUN = 0,
       PSNSHA = 0, T2MV = 0, Q2V = 0, CHV = 0, CHLEAF = 0, CHUC = 0, CHV2 = 0;
  real RSSUN = 0, RSSHA = 0, BGAP = 0, WGAP = 0;
  real UR = rmax(SQRT(UU * UU + VV * VV), K(1.0));
  real VAI = elai + esai;
  int VEG = (VAI > K(0.0));
  real FSNO = K(0.0);
  if (snowh > K(0.0)) {
    real BDSNO = sneqv / snowh;
    real FMELT = POW(BDSNO / K(100.0), (real)P->mltfct);
    FSNO = TANH(snowh / (K(2.5) * Z0 * FMELT));
  }
  real Z0MG;
  if (IST == 2) {
    if (TG <= TFRZ)
      Z0MG = K(0.01) * (K(1.0) - FSNO) + FSNO * (real)P->z0sno;
    else
      Z0MG = K(0.01);
  } else {
    Z0MG = Z0 * (K(1.0) - FSNO) + FSNO * (real)P->z0sno;
  }
  real ZPDG = snowh, Z0M, ZPD;
  if (VEG) {
    Z0M = VEGP(z0mvt);
    ZPD = K(0.65) * HTOP;
    if (snowh > ZPD) ZPD = snowh;
  } else {
    Z0M = Z0MG;
    ZPD = ZPDG;
  }
  real ZLVL = rmax(ZPD, HTOP) + ZREF;
  if (ZPDG >= ZLVL) ZLVL = ZPDG + ZREF;
  real CWP = VEGP(cwpvt);
  real DFb[7] = {0}, HCPCTb[7] = {0}, FACTb[7] = {0}, SNICEVb[3] = {0}, SNLIQVb[3] = {0},
       eporeb[3] = {0};
  real *DF = DFb + 2, *HCPCT = HCPCTb + 2, *FACT = FACTb + 2, *SNICEV = SNICEVb + 2,
       *SNLIQV = SNLIQVb + 2, *epore = eporeb + 2;
  thermoprop(X, sltyp, lutyp, ISNOW, IST, DZSNSO, DT, snowh, SNICE, SNLIQ, (real)P->csoil, SMC,
             soilwat, STC, DF, HCPCT, SNICEV, SNLIQV, epore, FACT);
  /* radiation: func.f90:1598-1714 */
  real ALBGRD[2], ALBGRI[2], ALBD[2], ALBI[2], FABD[2], FABI[2], FTDD[2], FTID[2], FTII[2];
  real FSUN, LAISUN, LAISHA, PARSUN, PARSHA, SAV, SAG, FSA, FSR;
  albedo(X, lutyp, IST, ISC, DT, COSZ, elai, esai, TG, TV, FSNO, FWET, SMC, SNEQVO, sneqv, QSNOW,
         fveg, &ALBOLD, &TAUSS, ALBGRD, ALBGRI, ALBD, ALBI, FABD, FABI, FTDD, FTID, FTII, &FSUN,
         &BGAP, &WGAP);
  real FSHA = K(1.0) - FSUN;
  LAISUN = elai * FSUN;
  LAISHA = elai * FSHA;
  real VAIr = elai + esai;
  surrad(K(1.0E-6), FSUN, FSHA, elai, VAIr, LAISUN, LAISHA, SOLAD, SOLAI, FABD, FABI, FTDD, FTID,
         FTII, ALBGRD, ALBGRI, ALBD, ALBI, &PARSUN, &PARSHA, &SAV, &SAG, &FSA, &FSR);
  real EMV = K(1.0) - EXP(-(elai + esai) / K(1.0));
  real EMG;
  if (ICE == 1)
    EMG = K(0.98) * (K(1.0) - FSNO) + K(1.0) * FSNO;
  else if (IST == 1)
    EMG = (real)P->emssoil * (K(1.0) - FSNO) + K(1.0) * FSNO;
  else
    EMG = (real)P->emslake * (K(1.0) - FSNO) + K(1.0) * FSNO;
  real BTRAN = K(0.0);
  const real PSIWLT = K(-150.);
  if (IST == 1) {
    for (int IZ = 1; IZ <= nroot; ++IZ) {
      real GX = K(0.0), PSI;
      if (O->opt_btr == 1)
        GX = (soilwat[IZ] - SOILP(smcwlt)) / (SOILP(smcref) - (SOILP(smcwlt)));
      if (O->opt_btr == 2) {
        PSI = rmax(PSIWLT,
                   -SOILP(psisat) * POW(rmax(K(0.01), soilwat[IZ]) / SOILP(smcmax), -SOILP(bexp)));
        GX = (K(1.0) - PSI / PSIWLT) / (K(1.0) + SOILP(psisat) / PSIWLT);
      }
      if (O->opt_btr == 3) {
        PSI = rmax(PSIWLT,
                   -SOILP(psisat) * POW(rmax(K(0.01), soilwat[IZ]) / SOILP(smcmax), -SOILP(bexp)));
        GX = K(1.0) - EXP(K(-5.8) * (LOG(PSIWLT / PSI)));
      }
      GX = rmin(K(1.0), rmax(K(0.0), GX));
      BTRANI[IZ] = rmax(MPE, DZSNSO[IZ] / (-ZSOIL[nroot]) * GX);
      BTRAN = BTRAN + BTRANI[IZ];
    }
    BTRAN = rmax(MPE, BTRAN);
    for (int IZ = 1; IZ <= nroot; ++IZ) BTRANI[IZ] = BTRANI[IZ] / BTRAN;
  }
  real RSURF, RHSUR;
  if (IST == 2) {
    RSURF = K(1.0);
    RHSUR = K(1.0);
  } else {
    real L_RSURF = (-ZSOIL[1]) *
                   (EXP(p5(K(1.0) - rmin(K(1.0), soilwat[1] / SOILP(smcmax)))) - K(1.0)) /
                   (K(2.71828) - K(1.0));
    real D_RSURF = K(2.2E-5) * SOILP(smcmax) * SOILP(smcmax) *
                   POW(K(1.0) - SOILP(smcwlt) / SOILP(smcmax), K(2.0) + K(3.0) / SOILP(bexp));
    RSURF = L_RSURF / D_RSURF;
    if (soilwat[1] < K(0.01) && snowh == K(0.0)) RSURF = K(1.0E6);
    real PSI = -SOILP(psisat) * POW(rmax(K(0.01), soilwat[1]) / SOILP(smcmax), -SOILP(bexp));
    RHSUR = FSNO + (K(1.0) - FSNO) * EXP(PSI * GRAV / (RVAP * TG));
  }
  if (lutyp == P->isurban && snowh == K(0.0)) RSURF = K(1.0E6);
  real LATHEAV, LATHEAG;
  int frozen_canopy, frozen_ground;
  if (TV > TFRZ) {
    LATHEAV = HVAP;
    frozen_canopy = 0;
  } else {
    LATHEAV = HSUB;
    frozen_canopy = 1;
  }
  real GAMMAV = CPAIR * SFCPRS / (K(0.622) * LATHEAV);
  if (TG > TFRZ) {
    LATHEAG = HVAP;
    frozen_ground = 0;
  } else {
    LATHEAG = HSUB;
    frozen_ground = 1;
  }
  real GAMMAG = CPAIR * SFCPRS / (K(0.622) * LATHEAG);
  real TGV = K(0.0), CMV = K(0.0);
  vegout_t vo;
  memset(&vo, 0, sizeof(vo));
  if (VEG && fveg > K(0.0)) {
    TGV = TG;
    CMV = CM;
    CHV = CH;
    vege_flux(X, ISNOW, lutyp, DT, SAV, SAG, LWDN, UR, UU, VV, SFCTMP, THAIR, QAIR, EAIR, RHOAIR,
              snowh, VAI, GAMMAV, GAMMAG, FWET, LAISUN, LAISHA, CWP, DZSNSO, HTOP, ZLVL, ZPD, Z0M,
              fveg, Z0MG, EMV, EMG, CANLIQ, CANICE, STC, DF, RSURF, LATHEAV, LATHEAG, PARSUN,
              PARSHA, IGS, FOLN, CO2AIR, O2AIR, BTRAN, SFCPRS, RHSUR, PSFC, &EAH, &TAH, &TV, &TGV,
              &CMV, &CHV, &QSFC, &vo);
    IRG = vo.IRG; IRC = vo.IRC; SHG = vo.SHG; SHC = vo.SHC; EVG = vo.EVG; EVC = vo.EVC;
    TR = vo.TR; GHV = vo.GH; T2MV = vo.T2MV; PSNSUN = vo.PSNSUN; PSNSHA = vo.PSNSHA;
    Q2V = vo.Q2V; CHV2 = vo.CAH2; CHLEAF = vo.CHLEAF; CHUC = vo.CHUC;
    RSSUN = vo.RSSUN; RSSHA = vo.RSSHA;
  }
  real TGB = TG, CMB = CM, CHB = CH;
  bareout_t bo;
  memset(&bo, 0, sizeof(bo));
  bare_flux(X, lutyp, ISNOW, SAG, LWDN, UR, UU, VV, SFCTMP, THAIR, QAIR, EAIR, RHOAIR, snowh,
            DZSNSO, ZLVL, ZPDG, Z0MG, EMG, STC, DF, RSURF, LATHEAG, GAMMAG, RHSUR, PSFC, &TGB,
            &CMB, &CHB, &QSFC, &bo);
  real FIRA, FSH, FGEV, SSOIL, FCEV, FCTR, T2M;
  if (VEG && fveg > K(0.0)) {
    FIRA = fveg * IRG + (K(1.0) - fveg) * bo.IRB + IRC;
    FSH = fveg * SHG + (K(1.0) - fveg) * bo.SHB + SHC;
    FGEV = fveg * EVG + (K(1.0) - fveg) * bo.EVB;
    SSOIL = fveg * GHV + (K(1.0) - fveg) * bo.GHB;
    FCEV = EVC;
    FCTR = TR;
    TG = fveg * TGV + (K(1.0) - fveg) * TGB;
    T2M = fveg * T2MV + (K(1.0) - fveg) * bo.T2MB;
    CM = fveg * CMV + (K(1.0) - fveg) * CMB;
    CH = fveg * CHV + (K(1.0) - fveg) * CHB;
  } else {
    FIRA = bo.IRB;
    FSH = bo.SHB;
    FGEV = bo.EVB;
    SSOIL = bo.GHB;
    TG = TGB;
    T2M = bo.T2MB;
    FCEV = K(0.);
    FCTR = K(0.);
    CM = CMB;
    CH = CHB;
    RSSUN = K(0.0);
    RSSHA = K(0.0);
    TGV = TGB;
    CHV = CHB;
  }
  real FIRE = LWDN + FIRA;
  if (FIRE <= K(0.0)) X->status |= NMP_ST_FIRE;
  real EMISSI = fveg * (EMG * (1 - EMV) + EMV + EMV * (1 - EMV) * (1 - EMG)) + (1 - fveg) * EMG;
  real TRAD = POW((FIRE - (K(1.0) - EMISSI) * LWDN) / (EMISSI * SB), K(0.25));
  real APAR = PARSUN * LAISUN + PARSHA * LAISHA;
  real PSN = PSNSUN * LAISUN + PSNSHA * LAISHA;
  tsnosoi(X, ISNOW, TBOT, ZSNSO, SSOIL, DF, HCPCT, (real)P->zbot, DT, snowh, STC);
  if (O->opt_stc == 2) {
    if (snowh > K(0.05) && TG > TFRZ) {
      TGV = TFRZ;
      TGB = TFRZ;
      if (VEG && fveg > K(0.0))
        TG = fveg * TGV + (K(1.0) - fveg) * TGB;
      else
        TG = TGB;
    }
  }
  real QMELT, PONDING;
  int IMELTb[7] = {0, 0, 0, 0, 0, 0, 0};
  int* IMELT = IMELTb + 2;
  phasechange(X, sltyp, ISNOW, DT, FACT, DZSNSO, IST, STC, SNICE, SNLIQ, &sneqv, &snowh, SMC,
              soilwat, &QMELT, IMELT, &PONDING);
  /* ===== end energy ===== */

  for (int k = 1; k <= NSOIL; ++k) soilice[k] = rmax(K(0.0), SMC[k] - soilwat[k]);
  SNEQVO = sneqv;
  real QVAP = rmax(FGEV / LATHEAG, K(0.0));
  real QDEW = FABS(rmin(FGEV / LATHEAG, K(0.0)));
  real EDIR = QVAP - QDEW;
  waterout_t wo;
  memset(&wo, 0, sizeof(wo));
  water(X, slptyp, sltyp, lutyp, DT, IMELT, UU, VV, FCEV, FCTR, QPRECC, QPRECL, elai, esai,
        SFCTMP, QVAP, QDEW, ZSOIL, BTRANI, FICEOLD, PONDING, TG, IST, fveg, frozen_canopy,
        frozen_ground, &ISNOW, &CANLIQ, &CANICE, &TV, &snowh, &sneqv, SNICE, SNLIQ, STC, ZSNSO,
        soilwat, SMC, soilice, &ZWT, &WA, &WT, DZSNSO, &WSLAKE, &FWET, &QSNOW, &wo);
  if (O->opt_veg == 2 || O->opt_veg == 5)
    carbon(P, lutyp, DT, ZSOIL, DZSNSO, STC, SMC, TV, PSN, FOLN, SOILP(smcmax), BTRAN, IGS,
           &LFMASS, &RTMASS, &STMASS, &WOOD, &STBLCP, &FASTCP, &GPP, &NPP, &NEE, &LAI, &SAI);
  /* error: func.f90:633-732 */
  real ERRSW = SWDOWN - (FSA + FSR);
  if (FABS(ERRSW) > K(0.01)) X->status |= NMP_ST_ERRSW;
  real ERRENG = SAV + SAG - (FIRA + FSH + FCEV + FGEV + FCTR + SSOIL);
  if (FABS(ERRENG) > K(0.01)) X->status |= NMP_ST_ERRENG;
  real QFX = wo.ETRAN + wo.ECAN + EDIR;
  real Q2B = bo.Q2B;
  if (lutyp == P->isurban) {
    QSFC = (QFX / RHOAIR * CH) + QAIR;
    Q2B = QSFC;
  }
  if (snowh <= K(1.0E-6) || sneqv <= K(1.0E-3)) {
    snowh = K(0.0);
    sneqv = K(0.0);
  }
  real ALBEDO = (SWDOWN != K(0.0)) ? FSR / SWDOWN : K(-999.9);

  /* pack */
  for (int k = 0; k < 7; ++k) {
    s[NMP_S_STC + k] = STCb[k];
    s[NMP_S_ZSNSO + k] = ZSNSOb[k];
  }
  for (int k = 0; k < 3; ++k) {
    s[NMP_S_SNICE + k] = SNICEb[k];
    s[NMP_S_SNLIQ + k] = SNLIQb[k];
  }
  for (int k = 1; k <= NSOIL; ++k) {
    s[NMP_S_SH2O + k - 1] = soilwat[k];
    s[NMP_S_SMC + k - 1] = SMC[k];
  }
  s[NMP_S_TV] = TV; s[NMP_S_TG] = TG; s[NMP_S_TAH] = TAH; s[NMP_S_EAH] = EAH;
  s[NMP_S_FWET] = FWET; s[NMP_S_CANLIQ] = CANLIQ; s[NMP_S_CANICE] = CANICE;
  s[NMP_S_QSFC] = QSFC; s[NMP_S_SNOWH] = snowh; s[NMP_S_SNEQV] = sneqv;
  s[NMP_S_SNEQVO] = SNEQVO; s[NMP_S_ALBOLD] = ALBOLD; s[NMP_S_TAUSS] = TAUSS;
  s[NMP_S_QSNOW] = QSNOW; s[NMP_S_ZWT] = ZWT; s[NMP_S_WA] = WA; s[NMP_S_WT] = WT;
  s[NMP_S_WSLAKE] = WSLAKE; s[NMP_S_LAI] = LAI; s[NMP_S_SAI] = SAI;
  s[NMP_S_LFMASS] = LFMASS; s[NMP_S_RTMASS] = RTMASS; s[NMP_S_STMASS] = STMASS;
  s[NMP_S_WOOD] = WOOD; s[NMP_S_STBLCP] = STBLCP; s[NMP_S_FASTCP] = FASTCP;
  s[NMP_S_CM] = CM; s[NMP_S_CH] = CH;
  *isnow_io = ISNOW;

  d[NMP_D_FSA] = FSA; d[NMP_D_FSR] = FSR; d[NMP_D_FIRA] = FIRA; d[NMP_D_FSH] = FSH;
  d[NMP_D_SSOIL] = SSOIL; d[NMP_D_FCEV] = FCEV; d[NMP_D_FGEV] = FGEV; d[NMP_D_FCTR] = FCTR;
  d[NMP_D_ECAN] = wo.ECAN; d[NMP_D_ETRAN] = wo.ETRAN; d[NMP_D_EDIR] = EDIR; d[NMP_D_TRAD] = TRAD;
  d[NMP_D_TGB] = TGB; d[NMP_D_TGV] = TGV; d[NMP_D_T2MV] = T2MV; d[NMP_D_T2MB] = bo.T2MB;
  d[NMP_D_Q2V] = Q2V; d[NMP_D_Q2B] = Q2B; d[NMP_D_RUNSRF] = wo.runsrf; d[NMP_D_RUNSUB] = wo.runsub;
  d[NMP_D_APAR] = APAR; d[NMP_D_PSN] = PSN; d[NMP_D_SAV] = SAV; d[NMP_D_SAG] = SAG;
  d[NMP_D_FSNO] = FSNO; d[NMP_D_NEE] = NEE; d[NMP_D_GPP] = GPP; d[NMP_D_NPP] = NPP;
  d[NMP_D_FVEG] = fveg; d[NMP_D_ALBEDO] = ALBEDO; d[NMP_D_QSNBOT] = wo.QSNBOT;
  d[NMP_D_PONDING] = PONDING; d[NMP_D_PONDING1] = wo.PONDING1; d[NMP_D_PONDING2] = wo.PONDING2;
  d[NMP_D_RSSUN] = RSSUN; d[NMP_D_RSSHA] = RSSHA; d[NMP_D_BGAP] = BGAP; d[NMP_D_WGAP] = WGAP;
  d[NMP_D_CHV] = CHV; d[NMP_D_CHB] = CHB; d[NMP_D_EMISSI] = EMISSI;
  d[NMP_D_SHG] = SHG; d[NMP_D_SHC] = SHC; d[NMP_D_SHB] = bo.SHB; d[NMP_D_EVG] = EVG;
  d[NMP_D_EVB] = bo.EVB; d[NMP_D_GHV] = GHV; d[NMP_D_GHB] = bo.GHB; d[NMP_D_IRG] = IRG;
  d[NMP_D_IRC] = IRC; d[NMP_D_IRB] = bo.IRB; d[NMP_D_TR] = TR; d[NMP_D_EVC] = EVC;
  d[NMP_D_CHLEAF] = CHLEAF; d[NMP_D_CHUC] = CHUC; d[NMP_D_CHV2] = CHV2; d[NMP_D_CHB2] = bo.EHB2;
  d[NMP_D_FPICE] = wo.FPICE;
  (void)T2M;
}

int oracle_real_bytes(void) { return (int)sizeof(real); }

int oracle_sflx_batch(int32_t n, real dt, int32_t yearlen, real julian, const real zsoil[4],
                      real* st, int32_t* isnow, const real* sf, const int32_t* si, const real* fc,
                      real* dg, int32_t* status, const nmp_params* P, const nmp_options* O) {
  for (int32_t c = 0; c < n; ++c) {
#ifdef ORACLE_ITER_STATS
    g_stat_col = c;
#endif
    ctx_t X = {P, O, 0};
    sflx_column(&X, dt, yearlen, julian, zsoil, st + (size_t)c * NMP_NSTATE, isnow + c,
                sf + (size_t)c * NMP_NSTATIC_F, si + (size_t)c * NMP_NSTATIC_I,
                fc + (size_t)c * NMP_NFORCING, dg + (size_t)c * NMP_NDIAG_FULL);
    status[c] = X.status;
  }
  return 0;
}

int oracle_sflx_run(int32_t n, int32_t nsteps, real dt, int32_t yearlen, real julian0,
                    const real zsoil[4], real* st, int32_t* isnow, const real* sf,
                    const int32_t* si, const real* fc, int32_t fc_period, real* dg,
                    int32_t* status, const nmp_params* P, const nmp_options* O) {
  for (int32_t s = 0; s < nsteps; ++s) {
    const real* f = fc + (size_t)(fc_period > 0 ? s % fc_period : 0) * n * NMP_NFORCING;
    real jul = julian0 + (real)s * dt / (real)86400.0;
    oracle_sflx_batch(n, dt, yearlen, jul, zsoil, st, isnow, sf, si, f, dg, status, P, O);
  }
  return 0;
}

/* ---- single routines, for the per-routine tests (tests/test_gpu_routines.py,
 * tests/test_oracle_golden.py): the same code sflx_column calls ---- */
void oracle_esat(int32_t n, const real* t, real* out4) {
  for (int32_t i = 0; i < n; ++i)
    esat(t[i], &out4[4 * i], &out4[4 * i + 1], &out4[4 * i + 2], &out4[4 * i + 3]);
}

void oracle_tdfcnd(const nmp_params* P, int32_t n, const int32_t* sltyp, const real* smc,
                   const real* sh2o, real* out) {
  for (int32_t i = 0; i < n; ++i) out[i] = tdfcnd(P, sltyp[i], smc[i], sh2o[i]);
}

void oracle_calhum(int32_t n, const real* sfctmp, const real* sfcprs, real* q2sat,
                   real* dqsdt2) {
  for (int32_t i = 0; i < n; ++i) calhum(sfctmp[i], sfcprs[i], &q2sat[i], &dqsdt2[i]);
}

void oracle_frh2o(const nmp_params* P, int32_t n, const int32_t* sltyp, const real* tk,
                  const real* smc, const real* sh2o, real* out, int32_t* status) {
  for (int32_t i = 0; i < n; ++i) {
    ctx_t X = {P, 0, 0};
    out[i] = frh2o(&X, sltyp[i], tk[i], smc[i], sh2o[i]);
    status[i] = X.status;
  }
}

/* one 7-layer system per column (layers -2..4 as 0..6), solved on layers
 * kt..6 (NTOP = kt in the 0-based storage); C is updated in place like the
 * reference's intent(inout) C */
void oracle_rosr12(int32_t n, const int32_t* kt, const real* a, const real* b, real* c,
                   const real* d, real* p, real* delta) {
  for (int32_t i = 0; i < n; ++i)
    rosr12(p + 7 * i, a + 7 * i, b + 7 * i, c + 7 * i, d + 7 * i, delta + 7 * i, kt[i], 6);
}
