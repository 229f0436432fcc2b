// Device routines of the sflx step that stand on their own, shared by the
// step kernel (sflx_kernel.hip) and the per-routine test library
// (tests/routines.hip), which checks each against the oracle's restatement
// and, for frh2o (the reference's one public routine), against the reference
// itself (tests/test_gpu_routines.py).
#pragma once
#include <hip/hip_runtime.h>

#include "dev_params.h"
#include "noahmp_engine.h"
#include "sflx_kargs.h"
#include "sflx_math.h"

namespace nmp {

// physical constants: core/module_noahmp_const.f90:14-35
#define MPE L(1.0E-6)
#define GRAV L(9.80616)
#define SB L(5.67E-8)
#define RGAS L(8.3144598)
#define KARMAN L(0.40)
#define TFRZ L(273.15)
#define HSUB L(2.8440E6)
#define HVAP L(2.5104E6)
#define HFUS L(0.3336E6)
#define CWAT L(4.188E6)
#define CICE L(2.094E6)
#define CPAIR L(1004.64)
#define TKWAT L(0.6)
#define TKICE L(2.2)
#define RAIR L(287.04)
#define RVAP L(461.269)
#define DENWAT L(1000.0)
#define DENICE L(917.0)

#define DEV __device__ __forceinline__

// ---------------------------------------------------------------------------
// esat: func.f90:3692-3736
template <class T>
DEV void esat(T t, T& esw, T& esi, T& desw, T& desi) {
  esw = L(100.) * (L(6.107799961) + t * (L(4.436518521E-01) + t * (L(1.428945805E-02) +
        t * (L(2.650648471E-04) + t * (L(3.031240396E-06) + t * (L(2.034080948E-08) +
        t * L(6.136820929E-11)))))));
  esi = L(100.) * (L(6.109177956) + t * (L(5.034698970E-01) + t * (L(1.886013408E-02) +
        t * (L(4.176223716E-04) + t * (L(5.824720280E-06) + t * (L(4.838803174E-08) +
        t * L(1.838826904E-10)))))));
  desw = L(100.) * (L(4.438099984E-01) + t * (L(2.857002636E-02) + t * (L(7.938054040E-04) +
         t * (L(1.215215065E-05) + t * (L(1.036561403E-07) + t * (L(3.532421810e-10) +
         t * L(-7.090244804E-13)))))));
  desi = L(100.) * (L(5.030305237E-01) + t * (L(3.773255020E-02) + t * (L(1.267995369E-03) +
         t * (L(2.477563108E-05) + t * (L(3.005693132E-07) + t * (L(2.158542548E-09) +
         t * L(7.131097725E-12)))))));
}

template <class T>
DEV T tdc(T t) { return rmin(L(50.0), rmax(L(-50.0), (t - TFRZ))); }

// The esat callers use (TT > 0) ? water : ice of each pair.  Evaluating only
// that pair behind a real branch (same expressions as esat) halves the work
// in waves whose lanes agree on the sign; mixed waves run both sides.
template <class T>
DEV void esat_sel(T t, T& es, T& des) {
  if (t > L(0.0)) {
    es = L(100.) * (L(6.107799961) + t * (L(4.436518521E-01) + t * (L(1.428945805E-02) +
         t * (L(2.650648471E-04) + t * (L(3.031240396E-06) + t * (L(2.034080948E-08) +
         t * L(6.136820929E-11)))))));
    des = L(100.) * (L(4.438099984E-01) + t * (L(2.857002636E-02) + t * (L(7.938054040E-04) +
          t * (L(1.215215065E-05) + t * (L(1.036561403E-07) + t * (L(3.532421810e-10) +
          t * L(-7.090244804E-13)))))));
  } else {
    es = L(100.) * (L(6.109177956) + t * (L(5.034698970E-01) + t * (L(1.886013408E-02) +
         t * (L(4.176223716E-04) + t * (L(5.824720280E-06) + t * (L(4.838803174E-08) +
         t * L(1.838826904E-10)))))));
    des = L(100.) * (L(5.030305237E-01) + t * (L(3.773255020E-02) + t * (L(1.267995369E-03) +
          t * (L(2.477563108E-05) + t * (L(3.005693132E-07) + t * (L(2.158542548E-09) +
          t * L(7.131097725E-12)))))));
  }
}
// value only (the derivative unused)
template <class T>
DEV T esat_val(T t) {
  if (t > L(0.0))
    return L(100.) * (L(6.107799961) + t * (L(4.436518521E-01) + t * (L(1.428945805E-02) +
           t * (L(2.650648471E-04) + t * (L(3.031240396E-06) + t * (L(2.034080948E-08) +
           t * L(6.136820929E-11)))))));
  return L(100.) * (L(6.109177956) + t * (L(5.034698970E-01) + t * (L(1.886013408E-02) +
         t * (L(4.176223716E-04) + t * (L(5.824720280E-06) + t * (L(4.838803174E-08) +
         t * L(1.838826904E-10)))))));
}

// NMP_UNFROZEN_FAST=0: no unfrozen-layer shortcuts (tdfcnd THKSAT, soilwater FCR):
// every layer through the powers and exponentials (A/B probe; results identical)
#ifndef NMP_UNFROZEN_FAST
#define NMP_UNFROZEN_FAST 1
#endif
// tdfcnd: func.f90:1500-1595
template <class T, bool R>
DEV T tdfcnd(const SoilRec& S, T smc, T sh2o) {
  typedef Mth<T, R> M;
  T smcmax = (T)S.smcmax, quartz = (T)S.quartz;
  T satratio = smc / smcmax;
  T thkw = L(0.57);
  T thkqtz = L(7.7);
  T xunfroz = sh2o / smc;
  T xu = xunfroz * smcmax;
  T thksat, thkdry;
  if constexpr (sizeof(T) == 4 && R) {
    // soil-type-only factors precomputed on the host (dev_params.h), bit-identical.
    // An unfrozen layer (SH2O == SMC, finite and positive) has XUNFROZ = 1 and
    // XU = SMCMAX exactly, so THKSAT is a soil-type constant too
    if (NMP_UNFROZEN_FAST && sh2o == smc && smc > L(0.0) && smc <= L(3.0e38))
      thksat = (T)S.tdf_thksat_wet;
    else
      thksat = (T)S.tdf_thks_pow * M::pow(TKICE, smcmax - xu) * M::pow(thkw, xu);
    thkdry = (T)S.tdf_thkdry;
  } else if constexpr (sizeof(T) == 8) {
    // fp64 (tolerance path): the type-only factors from the host in double, and
    // TKICE**(SMCMAX-XU) * THKW**XU as one exp with the logs of the constants
    thksat = (T)S.tdf_thks_pow_d *
             M::exp((smcmax - xu) * 0.7884573603642703 + xu * -0.5621189181535413);
    thkdry = (T)S.tdf_thkdry_d;
  } else {
    T thks = M::pow(thkqtz, quartz) * M::exp2(L(1.0) - quartz);  // 2.0**x -> exp2
    thksat = M::pow(thks, L(1.0) - smcmax) * M::pow(TKICE, smcmax - xu) * M::pow(thkw, xu);
    T gammd = (L(1.0) - smcmax) * L(2700.0);
    thkdry = (L(0.135) * gammd + L(64.7)) / (L(2700.0) - L(0.947) * gammd);
  }
  T ake;
  if ((sh2o + L(0.0005)) < smc)
    ake = satratio;
  else
    ake = (satratio > L(0.1)) ? M::log10(satratio) + L(1.0) : L(0.0);
  return ake * (thksat - thkdry) + thkdry;
}

// frh2o: func.f90:4494-4598 -- supercooled liquid water of a frozen soil
// layer (Koren et al. 1999), Newton iteration on the log form, with the
// Flerchinger explicit fallback (status bit) when it does not converge.
template <class T, bool R>
DEV T frh2o(T smcmax, T psisat, T bexp, T tkelv, T smc, T sh2o, int& status) {
  typedef Mth<T, R> M;
  T free_;
  T bx = bexp;
  if (bexp > L(5.5)) bx = L(5.5);
  if (tkelv > (TFRZ - L(1.0E-3))) {
    free_ = smc;
  } else {
    const T CK = L(8.0);
    T swl = smc - sh2o;
    if (swl > (smc - L(0.02))) swl = smc - L(0.02);
    if (swl < L(0.0)) swl = L(0.0);
    int nlog = 0, kcount = 0;
#pragma unroll 1
    while ((nlog < 10) && (kcount == 0)) {
      nlog = nlog + 1;
      T dfv = M::log((psisat * GRAV / HFUS) * p2(L(1.0) + CK * swl) *
                     M::pow(smcmax / (smc - swl), bx)) -
              M::log(-(tkelv - TFRZ) / tkelv);
      T den = L(2.0) * CK / (L(1.0) + CK * swl) + bx / (smc - swl);
      T swlk = swl - dfv / den;
      if (swlk > (smc - L(0.02))) swlk = smc - L(0.02);
      if (swlk < L(0.0)) swlk = L(0.0);
      T dswl = fabs(swlk - swl);
      swl = swlk;
      if (dswl <= L(0.005)) kcount = kcount + 1;
    }
    free_ = smc - swl;
    if (kcount == 0) {
      status |= NMP_ST_FLERCH;
      T fk = M::pow((HFUS / (GRAV * (-psisat))) * ((tkelv - TFRZ) / tkelv), L(-1.0) / bx) *
             smcmax;
      if (fk < L(0.02)) fk = L(0.02);
      free_ = rmin(fk, smc);
    }
  }
  return free_;
}

// calhum: func.f90:3958-3984 -- saturation mixing ratio (returned in g/g) and
// its temperature derivative.  The constant sub-expressions (ELWV/RV, 1./A3,
// A2*(A3-A4)) are folded by the reference's compiler in default real, which
// rounds exactly as these run-time operations do.
template <class T, bool R>
DEV void calhum(T sfctmp, T sfcprs, T& q2sat, T& dqsdt2) {
  typedef Mth<T, R> M;
  const T A2 = L(17.67), A3 = L(273.15), A4 = L(29.65), ELWV = L(2.501E6);
  const T A23M4 = A2 * (A3 - A4), E0 = L(0.611), RV = L(461.0), EPS = L(0.622);
  const T es = E0 * M::exp(ELWV / RV * (L(1.) / A3 - L(1.) / sfctmp));
  const T sfcprsx = sfcprs * L(1.E-3);
  q2sat = EPS * es / (sfcprsx - es);
  q2sat = q2sat * L(1.E3);
  dqsdt2 = (q2sat / (L(1.0) + q2sat)) * A23M4 / p2(sfctmp - A4);
  q2sat = q2sat / L(1.E3);
}

// rosr12 Thomas solve on layers kt..NL-1 (func.f90:4240-4288), static slots
template <class T, int NL>
DEV void rosr12(T (&p)[NL], const T (&a)[NL], const T (&b)[NL], T (&c)[NL], const T (&d)[NL],
                T (&delta)[NL], int kt) {
  c[NL - 1] = L(0.0);
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    if (k == kt) {
      p[k] = -c[k] / b[k];
      delta[k] = d[k] / b[k];
    } else if (k > kt) {
      const int km = k > 0 ? k - 1 : 0;
      p[k] = -c[k] * (L(1.0) / (b[k] + a[k] * p[km]));
      delta[k] = (d[k] - a[k] * delta[km]) * (L(1.0) / (b[k] + a[k] * p[km]));
    }
  }
  p[NL - 1] = delta[NL - 1];
#pragma unroll
  for (int k = NL - 2; k >= 0; --k)
    if (k >= kt) p[k] = p[k] * p[k + 1] + delta[k];
}

}  // namespace nmp
