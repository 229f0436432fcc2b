// Noah-MP column time step (noahmp_sflx) as one HIP kernel for gfx950.
//
// One lane owns one land column for the whole step: atm -> phenology ->
// energy (radiation, canopy/ground Newton iterations, snow/soil heat
// diffusion, phase change) -> water (canopy, snow layers, Richards,
// groundwater) -> carbon -> balance checks.  Reference:
// /root/reference/core/module_noahmp_func.f90 (line numbers in comments).
//
// MI355X mapping
//  - SoA field-major state in HBM: each of the 56 state fields, 12 forcing
//    fields and 12 static fields is one coalesced 256 B (fp32) wave load.
//  - Lookup tables (DevParams, ~9 KB) staged once per workgroup into LDS;
//    per-lane type lookups are ds_reads.
//  - Snow/soil layer arrays (7 layers) live in VGPRs: every layer loop is fully
//    unrolled over the 7 (or 3 / 4) static slots and predicated on the
//    column's active range, and the few truly dynamic subscripts (top layer
//    ISNOW+1, water-table layer) go through select chains (dget/dset), so no
//    array is ever demoted to scratch.
//  - Data-dependent Newton / bisection loops diverge per lane under the exec
//    mask; wave-uniform option branches become scalar branches.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dev_params.h"
#include "sflx_kargs.h"
#include "sflx_math.h"
#include "sflx_routines.h"
#include "vege_domain.h"

namespace nmp {

template <class T>
struct Col {
  // static
  int lutyp, sltyp, slptyp, isc, ist, ice;
  T lat, zref, shdfac, shdmax, tbot, foln;
  // forcing
  T sfctmp, sfcprs, psfc, uu, vv, q2, soldn, lwdn, prcp, cosz, co2air, o2air;
  // prognostic state
#ifdef NMP_LDS_STATE
  LArr<T, 7, 0> stc;
  LArr<T, 7, 7> zsnso;
  LArr<T, 3, 14> snice;
  LArr<T, 3, 17> snliq;
  LArr<T, 4, 20> sh2o;
  LArr<T, 4, 24> smc;
#else
  T stc[7], zsnso[7], snice[3], snliq[3], sh2o[4], smc[4];
#endif
  T tv, tg, tah, eah, fwet, canliq, canice, qsfc, snowh, sneqv, sneqvo, albold, tauss, qsnow;
  T zwt, wa, wt, wslake, lai, sai, lfmass, rtmass, stmass, wood, stblcp, fastcp, cm, ch;
  int isnow;
  // per-step layer work arrays
#ifdef NMP_LDS_WORK
  LArr<T, 7, 0> dz;
  LArr<T, 7, 7> df;
  LArr<T, 7, 14> hcpct;
  LArr<T, 7, 21> fact;
  T ficeold[3], sice[4], btrani[4];
#else
  T dz[7], ficeold[3], sice[4], btrani[4], df[7], hcpct[7], fact[7];
#endif
  int imelt[7];
  int status;
};

// twostream: func.f90:2215-2462 for one band / beam type
template <class T, bool R>
DEV void twostream_all(const DevParams& P, const VegRec& V, const Opt& o, T cosz, T vai, T fwet,
                       T t, const T (&albgrd)[2], const T (&albgri)[2], const T (&rho)[2],
                       const T (&tau)[2], T fveg, T (&fabd)[2], T (&albd)[2], T (&ftdd)[2],
                       T (&ftid)[2], T (&fabi)[2], T (&albi)[2], T (&ftii)[2], T& gdir, T& bgap,
                       T& wgap) {
  // twostream (func.f90:2215-2462) for both bands x both beams.  The reference
  // calls it 4 times; everything that does not depend on the band (crown gaps,
  // leaf-angle geometry, the avmu/asu log factors, exp(-ext*vai)) or on the
  // beam (h, s1, ...) is evaluated once here, with each expression's operand
  // order unchanged, so every output is bit-identical to the 4 separate calls.
  typedef Mth<T, R> M;
  const T PAI = L(3.14159265);
  T gap = L(0.0), kopen = L(0.0);
  if (vai == L(0.0)) {
    gap = L(1.0);
    kopen = L(1.0);
  } else {
    if (o.rad == 1) {
      T rc = (T)V.rcrown;
      T denfveg = -M::log(rmax(L(1.0) - fveg, L(0.01))) / (PAI * p2(rc));
      T hd = (T)V.hvt - (T)V.hvb;
      T bb = L(0.5) * hd;
      T thetap = M::atan(bb / rc * M::tan(M::acos(rmax(L(0.01), cosz))));
      bgap = M::exp(-denfveg * PAI * p2(rc) / M::cos(thetap));
      T fa = vai / (L(1.33) * PAI * p3(rc) * (bb / rc) * denfveg);
      T newvai = hd * fa;
      wgap = (L(1.0) - bgap) * M::exp(-L(0.5) * newvai / cosz);
      gap = rmin(L(1.0) - fveg, bgap + wgap);
      kopen = L(0.05);
    }
    if (o.rad == 2) {
      gap = L(0.0);
      kopen = L(0.0);
    }
    if (o.rad == 3) {
      gap = L(1.0) - fveg;
      kopen = L(1.0) - fveg;
    }
  }
  const T coszi = rmax(L(0.001), cosz);
  T chil = rmin(rmax((T)V.xl, L(-0.4)), L(0.6));
  if (fabs(chil) <= L(0.01)) chil = L(0.01);
  const T phi1 = L(0.5) - L(0.633) * chil - L(0.330) * chil * chil;
  const T phi2 = L(0.877) * (L(1.) - L(2.) * phi1);
  gdir = phi1 + phi2 * coszi;
  const T ext = gdir / coszi;
  const T avmu = (sizeof(T) == 4 && R) ? (T)V.avmu  // veg-type-only (dev_params.h)
                                       : (L(1.) - phi1 / phi2 * M::log((phi1 + phi2) / phi1)) / phi2;
  const T g_tmp0 = gdir + phi2 * coszi;
  const T g_tmp1 = phi1 * coszi;
  const T asu_f = (L(1.) - g_tmp1 / g_tmp0 * M::log((g_tmp1 + g_tmp0) / g_tmp1));
  const T chilf = p2((L(1.) + chil) / L(2.));
  const T s2 = M::exp(-ext * vai);
  const T avext = avmu * ext;
#pragma unroll
  for (int ib = 0; ib < 2; ++ib) {
    const T omegal = rho[ib] + tau[ib];
    const T asu = L(0.5) * omegal * gdir / g_tmp0 * asu_f;
    const T betadl = (L(1.) + avmu * ext) / (omegal * avmu * ext) * asu;
    const T betail = L(0.5) * (rho[ib] + tau[ib] + (rho[ib] - tau[ib]) * chilf) / omegal;
    T omega, betad, betai;
    if (t > TFRZ) {
      omega = omegal;
      betad = betadl;
      betai = betail;
    } else {
      const T oms = (T)P.g.omegas[ib];
      omega = (L(1.0) - fwet) * omegal + fwet * oms;
      betad = ((L(1.0) - fwet) * omegal * betadl + fwet * oms * (T)P.g.betads) / omega;
      betai = ((L(1.0) - fwet) * omegal * betail + fwet * oms * (T)P.g.betais) / omega;
    }
    const T b = L(1.) - omega + omega * betai;
    const T c = omega * betai;
    const T tmp0 = avext;
    const T d = tmp0 * omega * betad;
    const T f = tmp0 * omega * (L(1.) - betad);
    const T tmp1 = b * b - c * c;
    const T h = M::sqrt(tmp1) / avmu;
    T sigma = tmp0 * tmp0 - tmp1;
    if (fabs(sigma) < L(1.e-6)) sigma = copysign(L(1.e-6), sigma);
    const T p1 = b + avmu * h;
    const T pp2 = b - avmu * h;
    const T pp3 = b + tmp0;
    const T pp4 = b - tmp0;
    const T s1 = M::exp(-h * vai);
#pragma unroll
    for (int ic = 0; ic < 2; ++ic) {
      const T alb = (ic == 0) ? albgrd[ib] : albgri[ib];
      const T u1 = b - c / alb;
      const T u2 = b - c * alb;
      const T u3 = f + c * alb;
      const T tmp2 = u1 - avmu * h;
      const T tmp3 = u1 + avmu * h;
      const T d1 = p1 * tmp2 / s1 - pp2 * tmp3 * s1;
      const T tmp4 = u2 + avmu * h;
      const T tmp5 = u2 - avmu * h;
      const T d2 = tmp4 / s1 - tmp5 * s1;
      T ftd, fti, fre;
      if (ic == 0) {
        const T h1 = -d * pp4 - c * f;
        const T tmp6 = d - h1 * pp3 / sigma;
        const T tmp7 = (d - c - h1 / sigma * (u1 + tmp0)) * s2;
        const T h2 = (tmp6 * tmp2 / s1 - pp2 * tmp7) / d1;
        const T h3 = -(tmp6 * tmp3 * s1 - p1 * tmp7) / d1;
        const T h4 = -f * pp3 - c * d;
        const T tmp8 = h4 / sigma;
        const T tmp9 = (u3 - tmp8 * (u2 - tmp0)) * s2;
        const T h5 = -(tmp8 * tmp4 / s1 + tmp9) / d2;
        const T h6 = (tmp8 * tmp5 * s1 + tmp9) / d2;
        ftd = s2 * (L(1.0) - gap) + gap;
        fti = (h4 * s2 / sigma + h5 * s1 + h6 / s1) * (L(1.0) - gap);
        fre = (h1 / sigma + h2 + h3) * (L(1.0) - gap) + albgrd[ib] * gap;
      } else {
        const T h7 = (c * tmp2) / (d1 * s1);
        const T h8 = (-c * tmp3 * s1) / d1;
        const T h9 = tmp4 / (d2 * s1);
        const T h10 = (-tmp5 * s1) / d2;
        ftd = L(0.);
        fti = (h9 * s1 + h10 / s1) * (L(1.0) - kopen) + kopen;
        fre = (h7 + h8) * (L(1.0) - kopen) + albgri[ib] * kopen;
      }
      const T fab = L(1.0) - fre - (L(1.0) - albgrd[ib]) * ftd - (L(1.0) - albgri[ib]) * fti;
      if (ic == 0) {
        fabd[ib] = fab;
        albd[ib] = fre;
        ftdd[ib] = ftd;
        ftid[ib] = fti;
      } else {
        fabi[ib] = fab;
        albi[ib] = fre;
        ftii[ib] = fti;
      }
    }
  }
}

// sfcdif1: func.f90:3353-3508
// The four log terms of sfcdif1 (:3417-3420) depend only on heights fixed for
// the whole Newton loop; callers evaluate them once (same values, bit for bit)
// instead of once per iteration as the reference does.
template <class T, bool R>
struct Sfc1Logs {
  T tmpcm, tmpch, tmpcm2, tmpch2;
  DEV Sfc1Logs() : tmpcm(0), tmpch(0), tmpcm2(0), tmpch2(0) {}
  DEV Sfc1Logs(T zlvl, T zpd, T z0m, T z0h, int& status, const T* log_2z0m = nullptr) {
    typedef Mth<T, R> M;
    if (zlvl <= zpd) status |= NMP_ST_ZLVL;  // :3412-3415
    tmpcm = M::log((zlvl - zpd) / z0m);
    tmpch = (z0h == z0m) ? tmpcm : M::log((zlvl - zpd) / z0h);
    tmpcm2 = log_2z0m ? *log_2z0m : M::log((L(2.0) + z0m) / z0m);
    tmpch2 = (z0h == z0m) ? tmpcm2 : M::log((L(2.0) + z0h) / z0h);
  }
};

// The loop-invariant operands of sfcdif1's divisions (:3426-3432), formed
// once per loop by the caller through the loop's division policy `d`:
// KARMAN*(GRAV/TVIR), the reciprocal of RHOAIR*CPAIR, and the numerators
// ZLVL-ZPD and 2+Z0H (d.chk).  Same values, bit for bit, as forming them in
// every iteration as the reference does.
template <class T>
struct Sfc1Inv {
  T kgtv;          // KARMAN * (GRAV / TVIR)
  Recip<T> rhocp;  // RHOAIR * CPAIR
  T dz, d2;        // ZLVL - ZPD, 2 + Z0H
};
template <class T, class D>
DEV Sfc1Inv<T> sfc1_inv(D& d, T sfctmp, T qair, T rhoair, T zlvl, T zpd, T z0h) {
  const T tvir = (L(1.0) + L(0.61) * qair) * sfctmp;
  Sfc1Inv<T> v;
  v.kgtv = KARMAN * d.divk(GRAV, d.rec(tvir));
  v.rhocp = d.rec(rhoair * CPAIR);
  v.dz = zlvl - zpd;
  v.d2 = L(2.0) + z0h;
  d.chk(v.dz);
  d.chk(v.d2);
  return v;
}

template <class T, bool R, class D>
DEV void sfcdif1(D& d, const Sfc1Inv<T>& inv, int iter, T h, const Sfc1Logs<T, R>& lg, T ur,
                 T mpe, T& moz, int& mozsgn, T& fm, T& fh, T& fm2, T& fh2, T& cm, T& ch, T& fv,
                 bool two_m) {
  typedef Mth<T, R> M;
  T mozold = moz;
  const T tmpcm = lg.tmpcm, tmpch = lg.tmpch, tmpcm2 = lg.tmpcm2, tmpch2 = lg.tmpch2;
  T moz2;
  if (iter == 1) {
    fv = L(0.0);
    moz = L(0.0);
    moz2 = L(0.0);
  } else {
    T tmp1 = d.div(inv.kgtv * h, inv.rhocp);
    if (fabs(tmp1) <= mpe) tmp1 = mpe;
    const Recip<T> rmol = d.rec(d.div(L(-1.0) * p3(fv), d.rec(tmp1)));
    moz = rmin(d.divk(inv.dz, rmol), L(1.0));
    // the 2-m height's MOZ2 -> FM2/FH2 chain feeds only the 2-m diagnostics
    // (CHV2/CHB2 -> T2M, Q2): skipped when the step writes no diagnostics
    // (two_m false, wave-uniform), which changes no state value
    moz2 = two_m ? rmin(d.divk(inv.d2, rmol), L(1.0)) : L(0.0);
  }
  if (mozold * moz < L(0.0)) mozsgn = mozsgn + 1;
  if (mozsgn >= 2) {
    moz = L(0.0);
    fm = L(0.0);
    fh = L(0.0);
    moz2 = L(0.0);
    fm2 = L(0.0);
    fh2 = L(0.0);
  }
  T fmnew, fhnew, fm2new, fh2new;
  if (moz < L(0.0)) {
    T tmp1 = M::pow_q(L(1.0) - L(16.0) * moz);
    T tmp2 = M::log((L(1.0) + tmp1 * tmp1) / L(2.0));
    T tmp3 = M::log((L(1.0) + tmp1) / L(2.0));
    fmnew = L(2.0) * tmp3 + tmp2 - L(2.0) * M::atan(tmp1) + L(1.5707963);
    fhnew = L(2.0) * tmp2;
    if (two_m) {
      T tmp12 = M::pow_q(L(1.0) - L(16.0) * moz2);
      T tmp22 = M::log((L(1.0) + tmp12 * tmp12) / L(2.0));
      T tmp32 = M::log((L(1.0) + tmp12) / L(2.0));
      fm2new = L(2.0) * tmp32 + tmp22 - L(2.0) * M::atan(tmp12) + L(1.5707963);
      fh2new = L(2.0) * tmp22;
    } else {
      fm2new = fh2new = L(0.0);
    }
  } else {
    fmnew = L(-5.0) * moz;
    fhnew = fmnew;
    fm2new = L(-5.0) * moz2;
    fh2new = fm2new;
  }
  if (iter == 1) {
    fm = fmnew;
    fh = fhnew;
    fm2 = fm2new;
    fh2 = fh2new;
  } else {
    fm = L(0.5) * (fm + fmnew);
    fh = L(0.5) * (fh + fhnew);
    fm2 = L(0.5) * (fm2 + fm2new);
    fh2 = L(0.5) * (fh2 + fh2new);
  }
  fh = rmin(fh, L(0.9) * tmpch);
  fm = rmin(fm, L(0.9) * tmpcm);
  fh2 = rmin(fh2, L(0.9) * tmpch2);
  fm2 = rmin(fm2, L(0.9) * tmpcm2);
  T cmfm = tmpcm - fm;
  T chfh = tmpch - fh;
  T cm2fm2 = tmpcm2 - fm2;
  T ch2fh2 = tmpch2 - fh2;
  if (fabs(cmfm) <= mpe) cmfm = mpe;
  if (fabs(chfh) <= mpe) chfh = mpe;
  if (fabs(cm2fm2) <= mpe) cm2fm2 = mpe;
  if (fabs(ch2fh2) <= mpe) ch2fh2 = mpe;
  cm = d.divk(KARMAN * KARMAN, d.rec(cmfm * cmfm));
  ch = d.divk(KARMAN * KARMAN, d.rec(cmfm * chfh));
  fv = ur * d.sqrt(cm);  // CM in the proof's interval (tools/div_proof.py)
}

// sfcdif2 (Chen97, opt_sfc=2): func.f90:3511-3689
template <class T, bool R>
DEV void sfcdif2(int iter, T z0, T thz0, T thlm, T sfcspd, T czil, T zlm, T& akms, T& akhs,
                 T& rlmo, T& wstar2, T& ustar) {
  typedef Mth<T, R> M;
  const T WWST = L(1.2);
  const T WWST2 = WWST * WWST;
  const T VKRM = L(0.40), EXCM = L(0.001);
  const T BETA = L(1.0) / L(270.0);
  const T BTG = BETA * GRAV;
  const T ELFC = VKRM * BTG;
  const T WOLD = L(0.15);
  const T WNEW = L(1.0) - WOLD;
  const T PIHF = L(3.14159265) / L(2.);
  T zilfc = -czil * VKRM * L(258.2);
  T zu = z0;
  T rdz = L(1.0) / zlm;
  T cxch = EXCM * rdz;
  T dthv = thlm - thz0;
  T du2 = rmax(sfcspd * sfcspd, L(1.E-4));
  T btgh = BTG * L(1000.0);
  if (iter == 1) {
    if (btgh * akhs * dthv != L(0.0))
      wstar2 = WWST2 * M::pow(fabs(btgh * akhs * dthv), L(2.0) / L(3.0));
    else
      wstar2 = L(0.0);
    ustar = rmax(M::sqrt(akms * M::sqrt(du2 + wstar2)), L(0.07));
    rlmo = ELFC * akhs * dthv / p3(ustar);
  }
  T zt = rmax(L(1.0E-6), M::exp(zilfc * M::sqrt(ustar * z0)) * z0);
  T zslu = zlm + zu;
  T zslt = zlm + zt;
  T rlogu = M::log(zslu / zu);
  T rlogt = M::log(zslt / zt);
  T zetalt = rmax(zslt * rlmo, L(-5.0));
  rlmo = zetalt / zslt;
  T zetalu = zslu * rlmo;
  T zetau = zu * rlmo;
  T zetat = zt * rlmo;
  T simm, simh;
  if (rlmo < L(0.0)) {
    T xlu = M::sqrt(M::sqrt(L(1.0) - L(16.0) * zetalu));
    T xlt = M::sqrt(M::sqrt(L(1.0) - L(16.0) * zetalt));
    T xu = M::sqrt(M::sqrt(L(1.0) - L(16.0) * zetau));
    T xt = M::sqrt(M::sqrt(L(1.0) - L(16.0) * zetat));
    auto pspmu = [&](T xx) {
      return L(-2.0) * M::log((xx + L(1.0)) * L(0.5)) - M::log((xx * xx + L(1.0)) * L(0.5)) +
             L(2.0) * M::atan(xx) - PIHF;
    };
    auto psphu = [&](T xx) { return L(-2.0) * M::log((xx * xx + L(1.0)) * L(0.5)); };
    T psmz = pspmu(xu);
    simm = pspmu(xlu) - psmz + rlogu;
    T pshz = psphu(xt);
    simh = psphu(xlt) - pshz + rlogt;
  } else {
    zetalu = rmin(zetalu, L(1.0));
    zetalt = rmin(zetalt, L(1.0));
    T psmz = L(5.0) * zetau;
    simm = L(5.0) * zetalu - psmz + rlogu;
    T pshz = L(5.0) * zetat;
    simh = L(5.0) * zetalt - pshz + rlogt;
  }
  ustar = rmax(M::sqrt(akms * M::sqrt(du2 + wstar2)), L(0.07));
  zt = rmax(L(1.E-6), M::exp(zilfc * M::sqrt(ustar * z0)) * z0);
  zslt = zlm + zt;
  rlogt = M::log(zslt / zt);
  T ustark = ustar * VKRM;
  akms = rmax(ustark / simm, cxch);
  akhs = rmax(ustark / simh, cxch);
  if (btgh * akhs * dthv != L(0.0))
    wstar2 = WWST2 * M::pow(fabs(btgh * akhs * dthv), L(2.0) / L(3.0));
  else
    wstar2 = L(0.0);
  T rlmn = ELFC * akhs * dthv / p3(ustar);
  rlmo = rlmo * WOLD + rlmn * WNEW;
}

// ragrb: func.f90:3260-3350

// rhocp = d.rec(RHOAIR*CPAIR), rhcan = d.rec(HCAN) and dzg = ZPD-Z0MG
// (d.chk) are loop-invariant and formed once by the caller.
template <class T, bool R, class D>
DEV void ragrb(D& d, const Recip<T>& rhocp, const Recip<T>& rhcan, T dzg, T sqrt_dleaf_uc,
               int iter, T vai, T hg, T tah, T zpd, T z0hg, T hcan, T z0h, T fv, T cwp, T mpe,
               T& fhg, T& rahg, T& rb) {
  typedef Mth<T, R> M;
  T mozg = L(0.0);
  if (iter > 1) {
    T tmp1 = d.div(KARMAN * d.divk(GRAV, d.rec(tah)) * hg, rhocp);
    if (fabs(tmp1) <= mpe) tmp1 = mpe;
    const T molg = d.div(L(-1.) * p3(fv), d.rec(tmp1));
    mozg = rmin(d.divk(dzg, d.rec(molg)), L(1.0));
  }
  T fhgnew = (mozg < L(0.0)) ? M::pow_mq(L(1.0) - L(15.0) * mozg) : L(1.0) + L(4.7) * mozg;
  fhg = (iter == 1) ? fhgnew : L(0.5) * (fhg + fhgnew);
  T cwpc = d.sqrt(cwp * vai * hcan * fhg);  // proven range (tools/div_proof.py)
  T tmp1 = M::exp(d.div(-cwpc * z0hg, rhcan));
  T tmp2 = M::exp(d.div(-cwpc * (z0h + zpd), rhcan));
  T tmprah2 = d.div(hcan * M::exp(cwpc), d.rec(cwpc)) * (tmp1 - tmp2);
  T kh = rmax(KARMAN * fv * (hcan - zpd), mpe);
  rahg = d.div(tmprah2, d.rec(kh));
  T tmprb = d.div(cwpc * L(50.0), d.rec(L(1.0) - M::exp(-cwpc / L(2.0))));
  rb = tmprb * sqrt_dleaf_uc;
}

// stomata (Ball-Berry bisection): func.f90:3739-3887
// The sunlit and shaded calls (:2765-2770) share everything but APAR, so the
// APAR-independent prelude (:3829-3845: CF, KC, KO, AWC, CP, VCMX, RLB) is
// evaluated once (same expressions, bit-identical) and each call runs only
// its bisection.
template <class T>
struct StomataPre {
  T cf, kc, ko, awc, cp, vcmx, rlb;
  T fnf;  // MIN(FOLN / MAX(MPE, FOLNMX), 1) (the short-division domain check)
};

template <class T, bool R>
DEV StomataPre<T> stomata_pre(const VegRec& V, bool any_light, T sfcprs, T sfctmp, T tv, T o2,
                              T foln, T btran, T rb) {
  typedef Mth<T, R> M;
  StomataPre<T> p;
  p.cf = sfcprs / (RGAS * sfctmp) * L(1.0e06);
  p.kc = p.ko = p.awc = p.cp = p.vcmx = p.rlb = p.fnf = L(0.0);
  if (any_light) {
    T fnf = rmin(foln / rmax(MPE, (T)V.folnmx), L(1.0));
    p.fnf = fnf;
    T tc = tv - TFRZ;
    T ex = (tc - L(25.0)) / L(10.0);
    p.kc = (T)V.kc25 * M::pow((T)V.akc, ex);
    p.ko = (T)V.ko25 * M::pow((T)V.ako, ex);
    p.awc = p.kc * (L(1.0) + o2 / p.ko);
    p.cp = L(0.5) * p.kc / p.ko * o2 * L(0.21);
    p.vcmx = (T)V.vcmx25 /
             (L(1.0) + M::exp((L(-2.2E05) + L(710.0) * (tc + TFRZ)) / (L(8.314) * (tc + TFRZ)))) *
             fnf * btran * (M::pow((T)V.avcmx, ex));
    p.rlb = rb / p.cf;
  }
  return p;
}

template <class T, bool R, class D>
DEV void stomata_solve(D& d, const VegRec& V, const StomataPre<T>& p, T igs, T sfcprs, T apar,
                       T ea, T ei, T co2, T& rs, T& psn) {
  typedef Mth<T, R> M;
  const T CIERR = L(5.0E-2);
  const T cf = p.cf;
  rs = L(1.0) / (T)V.bp * cf;
  psn = L(0.0);
  if (apar <= L(0.0)) return;
  T ppf = L(4.6) * apar;
  T j = ppf * (T)V.qe25;
  const T kc = p.kc, awc = p.awc, cp = p.cp, vcmx = p.vcmx, rlb = p.rlb;
  (void)kc;
  T cihigh = L(1.5) * co2, cilow = L(0.0);
  const int c3c4 = V.c3c4;
  const T mp = (T)V.mp, bp = (T)V.bp;
#pragma unroll 1
  for (int iter = 1; iter <= 20; ++iter) {
    T ci = L(0.5) * (cihigh + cilow);
    T wc = (T)NAN, wj = (T)NAN, we = (T)NAN;  // SAVEd nan4 init (func.f90:3854-3856)
    if (c3c4 == 1) {
      wj = d.div(rmax(ci - cp, L(0.0)) * j, d.rec(ci + L(2.0) * cp));
      wc = d.div(rmax(ci - cp, L(0.0)) * vcmx, d.rec(ci + awc));
      we = L(0.5) * vcmx;
    } else if (c3c4 == 2) {
      wj = j;
      wc = vcmx;
      we = d.div(L(4000.0) * vcmx * ci, d.rec(sfcprs));
    }
    psn = rmin(rmin(wj, wc), we) * igs;
    T cs = rmax(co2 - L(1.37) * rlb * sfcprs * psn, MPE);
    T a = d.div(mp * psn * sfcprs * ea, d.rec(cs * ei)) + bp;
    T b = (d.div(mp * psn * sfcprs, d.rec(cs)) + bp) * rlb - L(1.0);
    T c = -rlb;
    T q = (b >= L(0.0)) ? L(-0.5) * (b + d.sqrt(b * b - L(4.0) * a * c))
                        : L(-0.5) * (b - d.sqrt(b * b - L(4.0) * a * c));
    T r1 = d.div(q, d.rec(a));
    T r2 = d.div(c, d.rec(q));
    rs = rmax(r1, r2);
    T fci = rmax(cs - psn * sfcprs * L(1.65) * rs, L(0.0));
    if (((cihigh - cilow) <= CIERR) || fabs(fci - ci) <= MPE) break;
    if (fci > ci)
      cilow = ci;
    else
      cihigh = ci;
  }
  rs = rs * cf;
}

// canres + calhum (Jarvis, opt_crs=2): func.f90:3890-3984
template <class T, bool R>
DEV void canres(const VegRec& V, T sfcprs, T tv, T par, T eah, T btran, T& rs, T& psn) {
  typedef Mth<T, R> M;
  T q2 = L(0.622) * eah / (sfcprs - L(0.378) * eah);
  q2 = q2 / (L(1.0) + q2);
  T q2sat, dqsdt2;  // (DQSDT2 unused by canres: the compiler drops it)
  calhum<T, R>(tv, sfcprs, q2sat, dqsdt2);
  T ff = L(2.0) * par / (T)V.rgl;
  T rcs = (ff + (T)V.rsmin / (T)V.rsmax) / (L(1.0) + ff);
  rcs = rmin(rmax(rcs, L(0.0001)), L(1.0));
  T rct = L(1.0) - L(0.0016) * p2((T)V.topt - tv);
  rct = rmin(rmax(rct, L(0.0001)), L(1.0));
  T rcq = L(1.0) / (L(1.0) + (T)V.hs * rmax(L(0.0), q2sat - q2));
  rcq = rmin(rmax(rcq, L(0.01)), L(1.0));
  rs = (T)V.rsmin / (rcs * rct * rcq * btran);
  psn = (T)NAN;
}

// combo: func.f90:5536-5577
template <class T>
DEV void combo(T& dz, T& wliq, T& wice, T& t, T dz2, T wliq2, T wice2, T t2) {
  T dzc = dz + dz2;
  T wicec = wice + wice2;
  T wliqc = wliq + wliq2;
  T h = (CICE * wice + CWAT * wliq) * (t - TFRZ) + HFUS * wliq;
  T h2 = (CICE * wice2 + CWAT * wliq2) * (t2 - TFRZ) + HFUS * wliq2;
  T hc = h + h2;
  T tc;
  if (hc < L(0.0))
    tc = TFRZ + hc / (CICE * wicec + CWAT * wliqc);
  else if (hc <= HFUS * wliqc)
    tc = TFRZ;
  else
    tc = TFRZ + (hc - HFUS * wliqc) / (CICE * wicec + CWAT * wliqc);
  dz = dzc;
  wice = wicec;
  wliq = wliqc;
  t = tc;
}

// combine: func.f90:5236-5413.  Snow slots j=0..2 <-> layers -2..0.
template <class T>
DEV void combine(Col<T>& c, T& ponding1, T& ponding2) {
  const int iso = c.isnow;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j >= iso + 3 && c.snice[j] <= L(0.1)) {
      if (j != 2) {
        const int j1 = j < 2 ? j + 1 : 2;
        c.snliq[j1] = c.snliq[j1] + c.snliq[j];
        c.snice[j1] = c.snice[j1] + c.snice[j];
      } else {
        if (iso < -1) {
          c.snliq[1] = c.snliq[1] + c.snliq[2];
          c.snice[1] = c.snice[1] + c.snice[2];
        } else {
          if (c.snice[2] >= L(0.0)) {
            ponding1 = c.snliq[2];
            c.sneqv = c.snice[2];
            c.snowh = c.dz[2];
          } else {
            ponding1 = c.snliq[2] + c.snice[2];
            if (ponding1 < L(0.0)) {
              c.sice[0] = rmax(L(0.0), c.sice[0] + ponding1 / (c.dz[3] * L(1000.0)));
              ponding1 = L(0.0);
            }
            c.sneqv = L(0.0);
            c.snowh = L(0.0);
          }
          c.snliq[2] = L(0.0);
          c.snice[2] = L(0.0);
          c.dz[2] = L(0.0);
        }
      }
      // shift the layers above down by one (J > ISNOW+1 .and. ISNOW < -1)
      if (j > c.isnow + 3 && c.isnow < -1) {
#pragma unroll
        for (int i = 2; i >= 1; --i) {
          if (i <= j && i >= c.isnow + 4) {  // Fortran I = J .. ISNOW+2
            c.stc[i] = c.stc[i - 1];
            c.snliq[i] = c.snliq[i - 1];
            c.snice[i] = c.snice[i - 1];
            c.dz[i] = c.dz[i - 1];
          }
        }
      }
      c.isnow = c.isnow + 1;
    }
  }
  if (c.sice[0] < L(0.0)) {
    c.sh2o[0] = c.sh2o[0] + c.sice[0];
    c.sice[0] = L(0.0);
  }
  if (c.isnow == 0) return;
  c.sneqv = L(0.0);
  c.snowh = L(0.0);
  T zwice = L(0.0), zwliq = L(0.0);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j >= c.isnow + 3) {
      c.sneqv = c.sneqv + c.snice[j] + c.snliq[j];
      c.snowh = c.snowh + c.dz[j];
      zwice = zwice + c.snice[j];
      zwliq = zwliq + c.snliq[j];
    }
  }
  if (c.snowh < L(0.025) && c.isnow < 0) {
    c.isnow = 0;
    c.sneqv = zwice;
    ponding2 = zwliq;
    if (c.sneqv <= L(0.0)) c.snowh = L(0.0);
  }
  if (c.isnow < -1) {
    const int iso2 = c.isnow;
    int mssi = 1;
    bool done = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (!done && i >= iso2 + 3) {
        const T dzmin = (mssi == 3) ? L(0.1) : L(0.025);
        if (c.dz[i] < dzmin) {
          // neighbour: I==ISNOW+1 -> I+1; I==0 -> I-1; else the thinner pair
          bool up;  // true: neighbour is i-1 (combine into slot i)
          if (i == 0)
            up = false;
          else if (i == 2)
            up = true;
          else
            up = (i == c.isnow + 3) ? false
                                    : ((c.dz[i - 1] + c.dz[i]) < (c.dz[i + 1] + c.dz[i]));
          if (!up) {  // J = i+1, L = i
            const int jj = i < 2 ? i + 1 : 2;
            combo(c.dz[jj], c.snliq[jj], c.snice[jj], c.stc[jj], c.dz[i], c.snliq[i], c.snice[i],
                  c.stc[i]);
#pragma unroll
            for (int k = 2; k >= 1; --k) {
              if (k <= jj - 1 && k >= c.isnow + 4) {  // Fortran K = J-1 .. ISNOW+2
                c.stc[k] = c.stc[k - 1];
                c.snice[k] = c.snice[k - 1];
                c.snliq[k] = c.snliq[k - 1];
                c.dz[k] = c.dz[k - 1];
              }
            }
          } else {  // J = i, L = i-1
            const int ll = i > 0 ? i - 1 : 0;
            combo(c.dz[i], c.snliq[i], c.snice[i], c.stc[i], c.dz[ll], c.snliq[ll], c.snice[ll],
                  c.stc[ll]);
#pragma unroll
            for (int k = 2; k >= 1; --k) {
              if (k <= i - 1 && k >= c.isnow + 4) {
                c.stc[k] = c.stc[k - 1];
                c.snice[k] = c.snice[k - 1];
                c.snliq[k] = c.snliq[k - 1];
                c.dz[k] = c.dz[k - 1];
              }
            }
          }
          c.isnow = c.isnow + 1;
          if (c.isnow >= -1) done = true;
        } else {
          mssi = mssi + 1;
        }
      }
    }
  }
}

// divide: func.f90:5416-5533
template <class T>
DEV void divide(Col<T>& c) {
  T dz[4] = {L(0.), L(0.), L(0.), L(0.)}, swice[4] = {L(0.), L(0.), L(0.), L(0.)};
  T swliq[4] = {L(0.), L(0.), L(0.), L(0.)}, tsno[4] = {L(0.), L(0.), L(0.), L(0.)};
  const int n = -c.isnow;
#pragma unroll
  for (int J = 1; J <= 3; ++J) {
    if (J <= n) {  // DZ(J) = DZSNSO(J+ISNOW): slot J+ISNOW+2
      const int s = J + c.isnow + 2;
      dz[J] = dget(c.dz, s);
      swice[J] = dget(c.snice, s);
      swliq[J] = dget(c.snliq, s);
      tsno[J] = dget(c.stc, s);
    }
  }
  int msno = n;
  if (msno == 1) {
    if (dz[1] > L(0.05)) {
      msno = 2;
      dz[1] = dz[1] / L(2.0);
      swice[1] = swice[1] / L(2.0);
      swliq[1] = swliq[1] / L(2.0);
      dz[2] = dz[1];
      swice[2] = swice[1];
      swliq[2] = swliq[1];
      tsno[2] = tsno[1];
    }
  }
  if (msno > 1) {
    if (dz[1] > L(0.05)) {
      T drr = dz[1] - L(0.05);
      T propor = drr / dz[1];
      T zwice = propor * swice[1];
      T zwliq = propor * swliq[1];
      propor = L(0.05) / dz[1];
      swice[1] = propor * swice[1];
      swliq[1] = propor * swliq[1];
      dz[1] = L(0.05);
      combo(dz[2], swliq[2], swice[2], tsno[2], drr, zwliq, zwice, tsno[1]);
      if (msno <= 2 && dz[2] > L(0.20)) {
        msno = 3;
        T dtdz = (tsno[1] - tsno[2]) / ((dz[1] + dz[2]) / L(2.));
        dz[2] = dz[2] / L(2.0);
        swice[2] = swice[2] / L(2.0);
        swliq[2] = swliq[2] / L(2.0);
        dz[3] = dz[2];
        swice[3] = swice[2];
        swliq[3] = swliq[2];
        tsno[3] = tsno[2] - dtdz * dz[2] / L(2.0);
        if (tsno[3] >= TFRZ)
          tsno[3] = tsno[2];
        else
          tsno[2] = tsno[2] + dtdz * dz[2] / L(2.0);
      }
    }
  }
  if (msno > 2) {
    if (dz[2] > L(0.2)) {
      T drr = dz[2] - L(0.2);
      T propor = drr / dz[2];
      T zwice = propor * swice[2];
      T zwliq = propor * swliq[2];
      propor = L(0.2) / dz[2];
      swice[2] = propor * swice[2];
      swliq[2] = propor * swliq[2];
      dz[2] = L(0.2);
      combo(dz[3], swliq[3], swice[3], tsno[3], drr, zwliq, zwice, tsno[2]);
    }
  }
  c.isnow = -msno;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j >= c.isnow + 3) {  // DZSNSO(J) = DZ(J-ISNOW): local index j-isnow-2
      const int s = j - c.isnow - 2;
      c.dz[j] = dget(dz, s);
      c.snice[j] = dget(swice, s);
      c.snliq[j] = dget(swliq, s);
      c.stc[j] = dget(tsno, s);
    }
  }
}

// ---------------------------------------------------------------------------
// noahmp_sflx for one column: func.f90:66-476
// layer thickness DZSNSO from the layer-bottom depths (func.f90:322-328)
template <class T>
DEV void layer_dz(Col<T>& c) {
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int km = k > 0 ? k - 1 : 0;
    if (k == c.isnow + 3)
      c.dz[k] = -c.zsnso[k];
    else if (k > c.isnow + 3)
      c.dz[k] = c.zsnso[km] - c.zsnso[k];
    else
      c.dz[k] = L(0.0);
  }
}

// Output sink: diagnostics and final state fields are written to HBM at the
// point they become final (not held in registers to the end of the step).
__host__ __device__ constexpr int out_index(int d) {
  return d == NMP_D_FSA ? NMP_O_FSA : d == NMP_D_FSR ? NMP_O_FSR : d == NMP_D_FIRA ? NMP_O_FIRA
       : d == NMP_D_FSH ? NMP_O_FSH : d == NMP_D_SSOIL ? NMP_O_SSOIL : d == NMP_D_FCEV ? NMP_O_FCEV
       : d == NMP_D_FGEV ? NMP_O_FGEV : d == NMP_D_FCTR ? NMP_O_FCTR : d == NMP_D_ECAN ? NMP_O_ECAN
       : d == NMP_D_ETRAN ? NMP_O_ETRAN : d == NMP_D_EDIR ? NMP_O_EDIR : d == NMP_D_TRAD ? NMP_O_TRAD
       : d == NMP_D_RUNSRF ? NMP_O_RUNSRF : d == NMP_D_RUNSUB ? NMP_O_RUNSUB
       : d == NMP_D_ALBEDO ? NMP_O_ALBEDO : -1;
}

// Streaming accesses of the column SoA (state, static, forcing, diagnostics):
// with the nontemporal hint (NMP_NT, default on), so that the once-read /
// once-written column data does not displace the register-spill lines from
// the XCD's L2: HBM traffic 903 -> 858 B per column-step, +0.5 % (config #3)
// and +0.9 % (config #5) (profiles/r02/nt_ab.txt).  NMP_NT=0: plain accesses.
#ifndef NMP_NT
#define NMP_NT 1
#endif
template <class T>
DEV T gld(const T* p) {
  if constexpr (NMP_NT != 0) return __builtin_nontemporal_load(p);
  else return *p;
}
template <class T>
DEV void gst(T* p, T v) {
  if constexpr (NMP_NT != 0) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Column addressing.  Every column array is field-major SoA with the
// launch's stride `ld`; element (field f, column c) of an array is at
// base + f*ld + c.  The bases are kernel arguments (SGPRs).  With NMP_OFF32
// the field's address base + f*ld stays uniform (SGPRs) and the lane adds
// one 32-bit VGPR, the byte offset c*sizeof(E), the same for every field: the
// SGPR-base + VGPR-offset form of global loads and stores (column indices
// below 2^29, which the host's argument checks guarantee).  NMP_OFF32=2
// also recomputes base + f*ld at every access (a few SALU instructions)
// rather than letting the compiler keep one live 64-bit base per field,
// which it spilled to VGPR lanes (94 SGPR spills, 700 v_readlane per step).
// NMP_OFF32=3 also re-reads the array base itself from the kernel-argument
// segment at each access (a scalar load) instead of holding the eight bases
// in SGPRs (892 -> 34 v_readlane).  Spilled VGPRs of the fp32 option-set-1
// kernel: 36 with 64-bit per-lane pointers (NMP_OFF32=0), 29 with 1, 9 with 2,
// 6 with 3.  Measured (profiles/r05/off32_ab.txt): 1 over 0 config #3 +1.8 %,
// config #5 +2.9 %; 2 over 1 +0.8 % and +3.3 %; 3 over 2 config #3 +2.1 %
// but config #5 -0.9 % and config #2 -6.8 % (fp64).  Default: 3 for the fp32
// translation unit, 2 for the fp64 one.
#ifndef NMP_OFF32
#if defined(NMP_TU) && NMP_TU == 4
#define NMP_OFF32 3
#else
#define NMP_OFF32 2
#endif
#endif
template <class E>
DEV E* col_at(E* base, int64_t ld, int64_t col, int f) {
  if constexpr (NMP_OFF32 != 0) {
#if NMP_OFF32 >= 2
    // an opaque copy of the stride per access: base + f*ld is formed here,
    // not shared with (and kept live for) the other accesses to field f
    __asm__ volatile("" : "+s"(ld));
#endif
    return (E*)((char*)(base + f * ld) + (uint32_t)((uint32_t)col * (uint32_t)sizeof(E)));
  } else
    return base + (f * ld + col);
}

#if NMP_OFF32 == 3
// the array bases re-read from the kernel-argument segment at every access
// (scalar loads) instead of being held in SGPRs: the step kernel's arguments
// are (const DevParams*, KArgs<T>), KArgs at byte offset 8 (the code object's
// .args metadata, which build.py check_kernarg_layout verifies for every
// sflx_step_kernel of each build; every kernel that uses Sink has this
// signature)
template <class T>
DEV const __attribute__((address_space(4))) KArgs<T>* kargs_seg() {
  const __attribute__((address_space(4))) char* p =
      (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
  __asm__ volatile("" : "+s"(p));
  return (const __attribute__((address_space(4))) KArgs<T>*)(p + 8);
}
#define NMP_KBASE(sink_member, karg_member) (kargs_seg<T>()->karg_member)
#else
#define NMP_KBASE(sink_member, karg_member) (sink_member)
#endif

template <class T>
struct Sink {
  T* dg;        // diag (column 0; NULL when level == NMP_DIAG_NONE)
  T* st;        // state (column 0)
  int64_t ld;
  int level;
  const T* sf;        // static_f (column 0)
  const int32_t* si;  // static_i (column 0)
  const T* fc;        // forcing (column 0)
  int32_t* isnow;     // isnow (column 0)
  uint8_t* cost;      // cost key (re-binning), or NULL
  const T* fice;      // caller FICEOLD, or NULL
  int64_t col;        // this lane's column
  template <class E>
  DEV E* at(E* base, int f) const { return col_at(base, ld, col, f); }
  // late loads: fields first needed deep in the step are read there, not at
  // kernel entry, so they do not hold registers through the energy phase
  DEV T ls(int f) const { return gld(at(NMP_KBASE(st, state), f)); }
  // state base laundered through an empty asm: loads through it are real
  // re-reads, never forwarded from values loaded earlier in the step
  DEV const T* fresh_state() const {
    const T* p = st;
    __asm__ volatile("" : "+s"(p));
    return p;
  }
  DEV T lf(int f) const { return gld(at(NMP_KBASE(sf, static_f), f)); }
  DEV int li(int f) const { return gld(at(NMP_KBASE(si, static_i), f)); }
  DEV T la(int f) const { return gld(at(NMP_KBASE(fc, forcing), f)); }
  template <int D>
  DEV void d(T v) const {
    if (level == NMP_DIAG_FULL) {
      gst(at(NMP_KBASE(dg, diag), D), v);
    } else if (level == NMP_DIAG_OUT) {
      constexpr int o = out_index(D);
      if (o >= 0) gst(at(NMP_KBASE(dg, diag), o), v);
    }
  }
  DEV void t2m(T v) const {
    if (level == NMP_DIAG_OUT) gst(at(NMP_KBASE(dg, diag), NMP_O_T2M), v);
  }
  DEV void s(int f, T v) const { gst(at(NMP_KBASE(st, state), f), v); }
  DEV void isn(int v) const { gst(at(NMP_KBASE(isnow, isnow), 0), (int32_t)v); }
  // re-binning key: the vege_flux Newton trip count of this step (0 = no canopy)
  DEV void trips(int n) const {
    if (cost) *at(cost, 0) = (uint8_t)n;
  }
};

// Layer-state copy in LDS (fp32 kernels): the 28 layer-state fields (STC,
// ZSNSO, SNICE, SNLIQ, SH2O, SMC = state fields 0..27) are copied HBM -> LDS
// at kernel entry by the load-to-LDS path (global_load_lds_dword, no VGPRs),
// read from there into registers for the energy phase, and read from there
// AGAIN after the flux loops instead of a second HBM read (the registers are
// not held through the loops, DESIGN.md "Layer state across the flux loops").
// Layout [field][thread] (28 x NMP_BLOCK floats, 28 KB per 256-thread block:
// with the 11.5 KB of tables four blocks still fit a CU's 160 KB).  Each lane
// reads back only its own slots, which its own wave's copy wrote, so no
// workgroup barrier is needed, only the wave's own wait for the DMA (an
// explicit s_waitcnt vmcnt(0) before the first read); nothing writes these
// fields before the second read.  (Issuing the
// copy later, as a prefetch before the flux loops, does not hide its latency:
// vmcnt counts in order, so the first spill reload after it waits for it.)
#ifndef NMP_PREFETCH
#define NMP_PREFETCH 3
#endif
// explicit wait for the copy before its first read (tuning A/B only: 0 leaves
// the wait to the compiler's LDS-DMA alias tracking, as round 2 did)
#ifndef NMP_LDS_EXPLICIT_WAIT
#define NMP_LDS_EXPLICIT_WAIT 1
#endif
constexpr int kPrefetchFields = NMP_S_SMC + 4;
static_assert(NMP_S_STC == 0 && NMP_S_ZSNSO == 7 && NMP_S_SNICE == 14 && NMP_S_SNLIQ == 17 &&
                  NMP_S_SH2O == 20 && NMP_S_SMC == 24,
              "prefetch slots are state fields 0..27");
template <class T, bool R>
constexpr bool kPrefetch = NMP_PREFETCH != 0 && sizeof(T) == 4 && R;
// (tuning: bit 0 = entry reads from the copy, bit 1 = the re-read from it)
template <class T, bool R>
constexpr bool kPfEntry = kPrefetch<T, R> && (NMP_PREFETCH & 1);
template <class T, bool R>
constexpr bool kPfReread = kPrefetch<T, R> && (NMP_PREFETCH & 2);
typedef __attribute__((address_space(3))) float lds_f32;
DEV lds_f32* lds_pool() {
  __shared__ float pool[kPrefetchFields * NMP_BLOCK];
  return (lds_f32*)pool;
}
template <class T>
DEV void copy_layers_to_lds(const T* st, int64_t ld) {
  lds_f32* pool = lds_pool();
  const int wbase = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63);
  // laundered base: the 28 field addresses are not shared with (and kept live
  // for) the step's other accesses to the same fields
  __asm__ volatile("" : "+v"(st));
#pragma unroll
  for (int f = 0; f < kPrefetchFields; ++f)
    __builtin_amdgcn_global_load_lds((const void*)(st + f * ld),
                                     (__attribute__((address_space(3))) void*)(pool + f * NMP_BLOCK + wbase),
                                     4, 0, NMP_NT != 0 ? 2 : 0);  // aux bit 1: nt
}

// Optional per-phase timing (build with -DNMP_PHASE_TIMING; tools only):
// each wave stamps s_memtime at phase boundaries and lane 0 accumulates the
// deltas into nmp_phase_cycles[phase].  Compiled out otherwise.
#ifdef NMP_PHASE_TIMING
static __device__ unsigned long long nmp_phase_cycles[16];
struct PhaseClock {
  unsigned long long t;
  int ph;
  DEV void mark(int next) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) atomicAdd(&nmp_phase_cycles[ph], now - t);
    t = now;
    ph = next;
  }
};
#define NMP_PHASE_MARK(i) pclk.mark(i)
#else
#define NMP_PHASE_MARK(i) ((void)0)
#endif
// Optional per-phase truncation (build with -DNMP_TRUNC_RUNTIME; tools only,
// tools/phase_counters.sh): the column's step returns at phase mark
// A.trunc_at (a kernel argument, so nothing before the mark is optimised
// away); consecutive marks' counters differ by one phase.
#ifdef NMP_TRUNC_RUNTIME
#define NMP_PHASE(i)                   \
  do {                                 \
    NMP_PHASE_MARK(i);                 \
    if (A.trunc_at == (i)) return;     \
  } while (0)
#else
#define NMP_PHASE(i) NMP_PHASE_MARK(i)
#endif

// Optional per-wave timing (build with -DNMP_WAVE_TIMING; tools only): each
// wave records {start, end} of s_memrealtime (100 MHz, one clock for the whole
// chip), its HW_ID/XCC_ID and {block, launch tag} into nmp_wave_rec, so that
// tools/wave_timeline.py can measure how full the wave slots stay over a launch
// (tail and workgroup-granularity idle time).  Compiled out otherwise.
#ifdef NMP_WAVE_TIMING
#define NMP_WAVE_REC_MAX (1 << 17)
static __device__ unsigned long long nmp_wave_rec[4 * NMP_WAVE_REC_MAX];
static __device__ unsigned int nmp_wave_ctr;
#endif
#ifdef NMP_COUNT_FALLBACK
static __device__ unsigned int nmp_fallback_ctr;
static __device__ unsigned int nmp_fb_reason[32];
#endif


// Unroll factor of the vege_flux Newton loop (tuning knob, results identical).
// NMP_VEGE_DIV: the canopy Newton loop divides with DivFast32 where its range
// proofs hold (fp32 "ref" option-set kernels), IEEE otherwise
#ifndef NMP_VEGE_DIV
#define NMP_VEGE_DIV 1
#endif
// NMP_BARE_DIV: the same for the bare-ground Newton loop (bare_flux)
#ifndef NMP_BARE_DIV
#define NMP_BARE_DIV 1
#endif
// NMP_SOIL_DIV: the soil-water sub-steps' divisions by the layer thicknesses
// (launch-uniform) with DivFast32, a tiny numerator on IEEE division
#ifndef NMP_SOIL_DIV
#define NMP_SOIL_DIV 1
#endif
// NMP_VD_CHECKED: bit 0 the canopy loop's CTR, TR and DTV, bit 1 the bare
// loop's DTG also divide with DivFast32, their numerators checked per lane
// every iteration (vege_domain.h NUM_LO_EXP / NUM_HI_EXP; outside: the lane
// re-runs its loop with IEEE division).  Both on: config #3 +0.4 to +1.4 %
// interleaved on two boxes, neither alone measurable
// (profiles/r06/ab/vd_checked_ab.txt)
#ifndef NMP_VD_CHECKED
#define NMP_VD_CHECKED 3
#endif
#ifndef NMP_VEGE_UNROLL
#define NMP_VEGE_UNROLL 1
#endif
// NMP_SKIP_2M=0: the 2-m diagnostic chain also on steps without diagnostics (A/B)
#ifndef NMP_SKIP_2M
#define NMP_SKIP_2M 1
#endif
// Unroll factors of the fixed 5-iteration under-canopy (loop2) and bare_flux
// Newton loops (tuning knobs, results identical).  bare_flux is unrolled in
// the fp32 kernels: config #3 +0.8 %, fewer spills (59 -> 52); fp64 and
// loop2 measured no gain (profiles/r02/unroll_ab.txt).
#ifndef NMP_LOOP2_UNROLL
#define NMP_LOOP2_UNROLL 1
#endif
#ifndef NMP_BARE_UNROLL
#define NMP_BARE_UNROLL sizeof(T) == 4 ? 5 : 1
#endif
// Late loads of the flux and water phases (fields first read there), issued
// where they are first needed (NMP_EARLY_LOADS=0) or a phase earlier, so
// that their memory latency overlaps the phase before (bit 1: water fields
// after the flux loops; bit 2: flux fields before btran/rsurf).  Values are
// the same either way: nothing stores these fields before the loads.
#ifndef NMP_EARLY_LOADS
#define NMP_EARLY_LOADS 0
#endif
#define NMP_FLUX_LOADS()                                                                     \
  c.tah = out.ls(NMP_S_TAH); c.eah = out.ls(NMP_S_EAH); c.canliq = out.ls(NMP_S_CANLIQ);     \
  c.canice = out.ls(NMP_S_CANICE); c.qsfc = out.ls(NMP_S_QSFC); c.cm = out.ls(NMP_S_CM);     \
  c.ch = out.ls(NMP_S_CH); c.tbot = out.lf(NMP_F_TBOT); c.foln = out.lf(NMP_F_FOLN);         \
  c.co2air = out.la(NMP_A_CO2AIR); c.o2air = out.la(NMP_A_O2AIR)
#define NMP_WATER_LOADS()                                                                    \
  const T prcp_w = out.la(NMP_A_PRCP), uu_w = out.la(NMP_A_UU), vv_w = out.la(NMP_A_VV);     \
  c.zwt = out.ls(NMP_S_ZWT); c.wa = out.ls(NMP_S_WA); c.wt = out.ls(NMP_S_WT);               \
  c.wslake = out.ls(NMP_S_WSLAKE);                                                           \
  c.slptyp = out.li(NMP_I_SLOPETYP)
#define NMP_STR(x) #x
#define NMP_UNROLL(n) _Pragma(NMP_STR(unroll n))

// Option sets compiled as constants (kernel template parameter OS): with the
// options known at compile time every `if (o.xxx == k)` of the other values
// folds away, which shortens the code and the live ranges of the hot loops.
// OS 0 reads the launch's options (every combination); 1 is run/case.nml's set
// (configs #1-#4), 2 the same with dynamic vegetation + carbon (opt_veg = 2,
// config #5).  The engine picks the set that matches its options.
constexpr Opt kOptionSet[3] = {{1, 1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1},
                               {1, 1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1},
                               {2, 1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1}};

template <class T, bool R, int OS>
DEV void sflx_column(const DevParams& P, const KArgs<T>& A, Col<T>& c, const Sink<T>& out) {
  typedef Mth<T, R> M;

#ifdef NMP_PHASE_TIMING
  PhaseClock pclk{__builtin_amdgcn_s_memtime(), 0};
#endif
  const Opt o = OS == 0 ? A.o : kOptionSet[OS];
  const VegRec& V = P.veg[c.lutyp - 1];
  const SoilRec& S = P.soil[c.sltyp - 1];
  const T DT = (T)A.dt;
  const T zsoil[4] = {(T)A.zsoil[0], (T)A.zsoil[1], (T)A.zsoil[2], (T)A.zsoil[3]};
  const T smcmax = (T)S.smcmax, smcwlt = (T)S.smcwlt, smcref = (T)S.smcref;
  const T bexp = (T)S.bexp, psisat = (T)S.psisat;
  const int nroot = V.nroot;

  // atm: func.f90:479-531
  T pair = c.sfcprs;
  // PAIR = SFCPRS: the ratio is exactly 1 for a finite nonzero pressure and
  // powf(1, y) = 1, so THAIR = SFCTMP * 1 = SFCTMP (other pressures: as written)
  T thair = (c.sfcprs != L(0.0) && fabs(c.sfcprs) <= L(3.0e38))
                ? c.sfctmp
                : c.sfctmp * M::pow(c.sfcprs / pair, RAIR / CPAIR);
  T qair = c.q2;
  T eair = qair * c.sfcprs / (L(0.622) + L(0.378) * qair);
  T rhoair = (c.sfcprs - L(0.378) * eair) / (RAIR * c.sfctmp);
  // QPRECC/QPRECL (:517-518) are only used by canwater: formed there from PRCP
  T swdown = (c.cosz <= L(0.0)) ? L(0.0) : c.soldn;
  T solad = swdown * L(0.7) * L(0.5);
  T solai = swdown * L(0.3) * L(0.5);

  // layer thickness (:322-328)
  layer_dz(c);
  // root-zone temperature (:332-335)
  T troot = L(0.0);
  {
    const T zr = -(nroot > 0 ? (T)zget(A.zsoil, nroot - 1) : L(1.0));
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nroot) troot = troot + c.stc[k + 3] * c.dz[k + 3] / zr;
  }

  // phenology: func.f90:534-630
  if (o.veg == 1 || o.veg == 3 || o.veg == 4) {
    T yl = (T)A.yearlen;
    T jul = (T)A.julian;
    T day = (c.lat >= L(0.0)) ? jul : fmod(jul + (L(0.5) * yl), yl);
    T t = L(12.0) * day / yl;
    int it1 = (int)(t + L(0.5));
    int it2 = it1 + 1;
    T wt1 = ((T)it1 + L(0.5)) - t;
    T wt2 = L(1.0) - wt1;
    if (it1 < 1) it1 = 12;
    if (it2 > 12) it2 = 1;
    c.lai = wt1 * (T)V.lai12m[it1 - 1] + wt2 * (T)V.lai12m[it2 - 1];
    c.sai = wt1 * (T)V.sai12m[it1 - 1] + wt2 * (T)V.sai12m[it2 - 1];
  }
  if (c.sai < L(0.05)) c.sai = L(0.0);
  if (c.lai < L(0.05) || c.sai == L(0.0)) c.lai = L(0.0);
  if (c.lutyp == P.g.iswater || c.lutyp == P.g.isbarren || c.lutyp == P.g.isice ||
      c.lutyp == P.g.isurban) {
    c.lai = L(0.0);
    c.sai = L(0.0);
  }
  // no carbon model: LAI/SAI are final here.  (Storing them before a
  // fast-division re-run is safe: for opt_veg 1/3/4 they are the table's
  // values above, whatever the stored ones were.)
  if (!(o.veg == 2 || o.veg == 5)) {
    out.s(NMP_S_LAI, c.lai);
    out.s(NMP_S_SAI, c.sai);
  }
  T elai, esai, igs, htop;
  {
    T hvt = (T)V.hvt, hvb = (T)V.hvb;
    T db = rmin(rmax(c.snowh - hvb, L(0.0)), hvt - hvb);
    T fb = db / rmax(L(1.0E-06), hvt - hvb);
    if (hvt > L(0.0) && hvt <= L(1.0)) {
      // no snow: EXP(-0) = 1 exactly (the exponential skipped)
      T snowhc = hvt * (c.snowh == L(0.0) ? L(1.0) : M::exp(-c.snowh / L(0.2)));
      fb = rmin(c.snowh, snowhc) / snowhc;
    }
    elai = c.lai * (L(1.0) - fb);
    esai = c.sai * (L(1.0) - fb);
    if (esai < L(0.05)) esai = L(0.0);
    if (elai < L(0.05) || esai == L(0.0)) elai = L(0.0);
    igs = (c.tv > (T)V.tmin) ? L(1.0) : L(0.0);
    htop = hvt;
  }
  // vegetation fraction (:366-380)
  T fveg = L(0.0);
  if (o.veg == 1) {
    fveg = c.shdfac;
    if (fveg <= L(0.01)) fveg = L(0.01);
  } else if (o.veg == 2 || o.veg == 3) {
    fveg = L(1.0) - M::exp(L(-0.52) * (c.lai + c.sai));
    if (fveg <= L(0.01)) fveg = L(0.01);
  } else if (o.veg == 4 || o.veg == 5) {
    fveg = c.shdmax;
    if (fveg <= L(0.01)) fveg = L(0.01);
  } else {
    c.status |= NMP_ST_OPTVEG;
  }
  if (c.lutyp == P.g.isurban || c.lutyp == P.g.isbarren) fveg = L(0.0);
  if (elai + esai == L(0.0)) fveg = L(0.0);

  // ===================== energy: func.f90:735-1338 =====================
  const T Z0 = L(0.01);
  const int kt = c.isnow + 3;  // top active layer slot
  T irc = 0, shc = 0, irg = 0, shg = 0, evg = 0, evc = 0, tr = 0, ghv = 0, psnsun = 0, psnsha = 0;
  T t2mv = 0, q2v = 0, chv = 0, chleaf = 0, chuc = 0, chv2 = 0, rssun = 0, rssha = 0;
  // the diagnostic-only chains (the 2-m MOZ2 -> FH2 -> CHV2/CHB2 -> T2M, Q2;
  // TRAD) only when the step writes diagnostics: nothing else reads them
  const bool diag_on = !NMP_SKIP_2M || out.level != NMP_DIAG_NONE;
  T bgap = 0, wgap = 0;
  T ur = rmax(M::sqrt(c.uu * c.uu + c.vv * c.vv), L(1.0));
  T vai = elai + esai;
  const bool veg = vai > L(0.0);
  T fsno = L(0.0);
  if (c.snowh > L(0.0)) {
    T bdsno = c.sneqv / c.snowh;
    T fmelt = M::pow(bdsno / L(100.0), (T)P.g.mltfct);
    fsno = M::tanh(c.snowh / (L(2.5) * Z0 * fmelt));
  }
  T z0mg;
  if (c.ist == 2)
    z0mg = (c.tg <= TFRZ) ? L(0.01) * (L(1.0) - fsno) + fsno * (T)P.g.z0sno : L(0.01);
  else
    z0mg = Z0 * (L(1.0) - fsno) + fsno * (T)P.g.z0sno;
  T zpdg = c.snowh, z0m, zpd;
  if (veg) {
    z0m = (T)V.z0mvt;
    zpd = L(0.65) * htop;
    if (c.snowh > zpd) zpd = c.snowh;
  } else {
    z0m = z0mg;
    zpd = zpdg;
  }
  T zlvl = rmax(zpd, htop) + c.zref;
  if (zpdg >= zlvl) zlvl = zpdg + c.zref;
  const T cwp = (T)V.cwpvt;

  NMP_PHASE(1);
  // Top-layer conductivity DF(ISNOW+1) for the flux Newton loops, computed
  // exactly as thermoprop computes that element (full thermoprop runs after
  // the fluxes, so its 21 layer values are not held through the iterations).
  T df_top;
  if (kt < 3) {  // snow top layer: csnow (:1490)
    const T sn_ice = dget(c.snice, kt), sn_liq = dget(c.snliq, kt), sn_dz = dget(c.dz, kt);
    const T bdsnoi = (sn_ice + sn_liq) / sn_dz;
    df_top = L(3.2217E-6) * p2(bdsnoi);
  } else {  // soil layer 1 + snow/soil interface (:1400-1444)
    T df3 = tdfcnd<T, R>(S, c.smc[0], c.sh2o[0]);
    if (c.lutyp == P.g.isurban) df3 = L(3.24);
    if (c.ist == 2) df3 = (c.stc[3] > TFRZ) ? TKWAT : TKICE;
    df_top = (df3 * c.dz[3] + L(0.35) * c.snowh) / (c.snowh + c.dz[3]);
  }

  NMP_PHASE(2);
  // radiation: albedo + twostream + surrad (func.f90:1598-2005)
  T albgrd[2] = {L(0.), L(0.)}, albgri[2] = {L(0.), L(0.)}, albd[2] = {L(0.), L(0.)};
  T albi[2] = {L(0.), L(0.)}, fabd[2] = {L(0.), L(0.)}, fabi[2] = {L(0.), L(0.)};
  T ftdd[2] = {L(0.), L(0.)}, ftid[2] = {L(0.), L(0.)}, ftii[2] = {L(0.), L(0.)};
  T fsun = L(0.0);
  if (c.cosz > L(0.0)) {
    // snow-age / albedo state is only read and updated in daylight (:1823):
    // load it here, store it at the end of this block
    c.albold = out.ls(NMP_S_ALBOLD); c.tauss = out.ls(NMP_S_TAUSS);
    c.qsnow = out.ls(NMP_S_QSNOW); c.sneqvo = out.ls(NMP_S_SNEQVO);
    const T mpe6 = L(1.0E-06);
    T rho[2], tau[2];
    T vaia = elai + esai;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      T wl = elai / rmax(vaia, mpe6);
      T ws = esai / rmax(vaia, mpe6);
      rho[ib] = rmax((T)V.rhol[ib] * wl + (T)V.rhos[ib] * ws, mpe6);
      tau[ib] = rmax((T)V.taul[ib] * wl + (T)V.taus[ib] * ws, mpe6);
    }
    // snowage: func.f90:2008-2054
    T fage;
    if (c.sneqv <= L(0.0)) {
      c.tauss = L(0.0);
    } else if (c.sneqv > L(800.0)) {
      c.tauss = L(0.0);
    } else {
      T dela0 = L(1.0E-6) * DT;
      T arg = L(5.0E3) * (L(1.0) / TFRZ - L(1.0) / c.tg);
      T age1 = M::exp(arg);
      T age2 = M::exp(rmin(L(0.0), L(10.0) * arg));
      T tage = age1 + age2 + L(0.3);
      T dela = dela0 * tage;
      T dels = rmax(L(0.0), c.sneqv - c.sneqvo) / (T)P.g.swemax;
      T sge = (c.tauss + dela) * (L(1.0) - dels);
      c.tauss = rmax(L(0.0), sge);
    }
    fage = c.tauss / (c.tauss + L(1.0));
    T albsnd[2] = {L(0.), L(0.)}, albsni[2] = {L(0.), L(0.)};
    if (o.alb == 1) {  // snowalb_bats: func.f90:2057-2102
      T sl = L(2.0);
      T sl1 = L(1.0) / sl;
      T sl2 = L(2.0) * sl;
      T cf1 = ((L(1.0) + sl1) / (L(1.0) + sl2 * c.cosz) - sl1);
      T fzen = rmax(cf1, L(0.0));
      albsni[0] = L(0.95) * (L(1.0) - L(0.2) * fage);
      albsni[1] = L(0.65) * (L(1.0) - L(0.5) * fage);
      albsnd[0] = albsni[0] + L(0.4) * fzen * (L(1.0) - albsni[0]);
      albsnd[1] = albsni[1] + L(0.4) * fzen * (L(1.0) - albsni[1]);
    }
    if (o.alb == 2) {  // snowalb_class: func.f90:2105-2151
      const T decay = (sizeof(T) == 4 && R) ? (T)A.c_albdecay : M::exp(-L(0.01) * DT / L(3600.0));
      T alb = L(0.55) + (c.albold - L(0.55)) * decay;
      if (c.qsnow > L(0.0))
        alb = alb + rmin(c.qsnow * DT, (T)P.g.swemax) * (L(0.84) - alb) / (T)P.g.swemax;
      albsnd[0] = albsnd[1] = albsni[0] = albsni[1] = alb;
      c.albold = alb;
    }
    // groundalb: func.f90:2154-2212
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      T inc = rmax(L(0.11) - L(0.40) * c.smc[0], L(0.0));
      T albsod, albsoi;
      if (c.ist == 1) {
        albsod = rmin((T)P.g.albsat[c.isc - 1][ib] + inc, (T)P.g.albdry[c.isc - 1][ib]);
        albsoi = albsod;
      } else if (c.tg > TFRZ) {
        albsod = L(0.06) / (M::pow(rmax(L(0.01), c.cosz), L(1.7)) + L(0.15));
        albsoi = L(0.06);
      } else {
        albsod = (T)P.g.alblake[ib];
        albsoi = albsod;
      }
      if (c.ist == 1 && c.isc == 9) {
        albsod = albsod + L(0.10);
        albsoi = albsoi + L(0.10);
      }
      albgrd[ib] = albsod * (L(1.0) - fsno) + albsnd[ib] * fsno;
      albgri[ib] = albsoi * (L(1.0) - fsno) + albsni[ib] * fsno;
    }
    T gdir = L(0.0);
    twostream_all<T, R>(P, V, o, c.cosz, vaia, c.fwet, c.tv, albgrd, albgri, rho, tau, fveg, fabd,
                        albd, ftdd, ftid, fabi, albi, ftii, gdir, bgap, wgap);
    T ext = gdir / c.cosz * M::sqrt(L(1.0) - rho[0] - tau[0]);
    fsun = (L(1.0) - M::exp(-ext * vaia)) / rmax(ext * vaia, mpe6);
    ext = fsun;
    fsun = (ext < L(0.01)) ? L(0.) : ext;
    out.s(NMP_S_ALBOLD, c.albold);
    out.s(NMP_S_TAUSS, c.tauss);
  }
  T fsha = L(1.0) - fsun;
  T laisun = elai * fsun;
  T laisha = elai * fsha;
  T sav, sag, fsa, fsr, parsun, parsha;
  {
    T cad0 = solad * fabd[0], cai0 = solai * fabi[0];
    T cad1 = solad * fabd[1], cai1 = solai * fabi[1];
    sag = L(0.0);
    sav = L(0.0);
    fsa = L(0.0);
    sav = sav + cad0 + cai0;
    fsa = fsa + cad0 + cai0;
    T abs0 = (solad * ftdd[0]) * (L(1.0) - albgrd[0]) +
             (solad * ftid[0] + solai * ftii[0]) * (L(1.0) - albgri[0]);
    sag = sag + abs0;
    fsa = fsa + abs0;
    sav = sav + cad1 + cai1;
    fsa = fsa + cad1 + cai1;
    T abs1 = (solad * ftdd[1]) * (L(1.0) - albgrd[1]) +
             (solad * ftid[1] + solai * ftii[1]) * (L(1.0) - albgri[1]);
    sag = sag + abs1;
    fsa = fsa + abs1;
    T laifra = elai / rmax(vai, L(1.0E-6));
    if (fsun > L(0.0)) {
      parsun = (cad0 + fsun * cai0) * laifra / rmax(laisun, L(1.0E-6));
      parsha = (fsha * cai0) * laifra / rmax(laisha, L(1.0E-6));
    } else {
      parsun = L(0.0);
      parsha = (cad0 + cai0) * laifra / rmax(laisha, L(1.0E-6));
    }
    fsr = (albd[0] * solad + albi[0] * solai) + (albd[1] * solad + albi[1] * solai);
  }
  if (fabs(swdown - (fsa + fsr)) > L(0.01)) c.status |= NMP_ST_ERRSW;  // error() :688-710
  out.template d<NMP_D_FSA>(fsa);
  out.template d<NMP_D_FSR>(fsr);
  out.template d<NMP_D_ALBEDO>((swdown != L(0.0)) ? fsr / swdown : L(-999.9));  // :470-474
  out.template d<NMP_D_FSNO>(fsno);
  out.template d<NMP_D_FVEG>(fveg);
  out.template d<NMP_D_BGAP>(bgap);
  out.template d<NMP_D_WGAP>(wgap);
  // no leaves or stems: EXP(-0) = 1 and EMV = +0 exactly (the exponential skipped)
  T emv = (elai + esai == L(0.0)) ? L(0.0) : L(1.0) - M::exp(-(elai + esai) / L(1.0));
  T emg;
  if (c.ice == 1)
    emg = L(0.98) * (L(1.0) - fsno) + L(1.0) * fsno;
  else if (c.ist == 1)
    emg = (T)P.g.emssoil * (L(1.0) - fsno) + L(1.0) * fsno;
  else
    emg = (T)P.g.emslake * (L(1.0) - fsno) + L(1.0) * fsno;
  NMP_PHASE(3);
#if NMP_EARLY_LOADS & 2
  // the flux phase's fields issued here, their latency under btran/rsurf
  NMP_FLUX_LOADS();
#endif
  // soil moisture stress (:1117-1140)
  T btran = L(0.0);
#pragma unroll
  for (int k = 0; k < 4; ++k) c.btrani[k] = L(0.0);
  if (c.ist == 1) {
    const T zr = -(nroot > 0 ? (T)zget(A.zsoil, nroot - 1) : L(1.0));
    const T PSIWLT = L(-150.);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < nroot) {
        T gx = L(0.0);
        if (o.btr == 1) gx = (c.sh2o[k] - smcwlt) / (smcref - (smcwlt));
        if (o.btr == 2 || o.btr == 3) {
          T psi = rmax(PSIWLT, -psisat * M::pow(rmax(L(0.01), c.sh2o[k]) / smcmax, -bexp));
          if (o.btr == 2)
            gx = (L(1.0) - psi / PSIWLT) / (L(1.0) + psisat / PSIWLT);
          else
            gx = L(1.0) - M::exp(L(-5.8) * (M::log(PSIWLT / psi)));
        }
        gx = rmin(L(1.0), rmax(L(0.0), gx));
        c.btrani[k] = rmax(MPE, c.dz[k + 3] / zr * gx);
        btran = btran + c.btrani[k];
      }
    }
    btran = rmax(MPE, btran);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nroot) c.btrani[k] = c.btrani[k] / btran;
  }
  // ground surface resistance (:1143-1169)
  T rsurf, rhsur;
  if (c.ist == 2) {
    rsurf = L(1.0);
    rhsur = L(1.0);
  } else {
    T l_rsurf = (-zsoil[0]) * (M::exp(p5(L(1.0) - rmin(L(1.0), c.sh2o[0] / smcmax))) - L(1.0)) /
                (L(2.71828) - L(1.0));
    T d_rsurf = (sizeof(T) == 4 && R) ? (T)S.rsurf_den  // soil-type-only (dev_params.h)
                                      : L(2.2E-5) * smcmax * smcmax *
                                            M::pow(L(1.0) - smcwlt / smcmax, L(2.0) + L(3.0) / bexp);
    rsurf = l_rsurf / d_rsurf;
    if (c.sh2o[0] < L(0.01) && c.snowh == L(0.0)) rsurf = L(1.0E6);
    T psi = -psisat * M::pow(rmax(L(0.01), c.sh2o[0]) / smcmax, -bexp);
    rhsur = fsno + (L(1.0) - fsno) * M::exp(psi * GRAV / (RVAP * c.tg));
  }
  if (c.lutyp == P.g.isurban && c.snowh == L(0.0)) rsurf = L(1.0E6);
  const bool frozen_canopy = !(c.tv > TFRZ);
  T latheav = frozen_canopy ? HSUB : HVAP;
  T gammav = CPAIR * c.sfcprs / (L(0.622) * latheav);
  const bool frozen_ground = !(c.tg > TFRZ);
  const T latheag = frozen_ground ? HSUB : HVAP;
  const T gammag = CPAIR * c.sfcprs / (L(0.622) * latheag);
  const T stc_top = dget(c.stc, kt), dz_top = dget(c.dz, kt);

  // fields first used by the flux phase
#if !(NMP_EARLY_LOADS & 2)
  NMP_FLUX_LOADS();
#endif
  NMP_PHASE(4);
// NMP_DOM_MASK (timing probes only, not exact in general): the checks kept
#ifndef NMP_DOM_MASK
#define NMP_DOM_MASK 0xffffffffu
#endif
#ifdef NMP_COUNT_FALLBACK
  // (probe builds) which condition sent the lane to an IEEE loop
  unsigned fb_why = 0;
#define NMP_DOM(flag, bit, cond)                 \
  do {                                           \
    const bool c_ = (cond);                      \
    flag = flag & c_;                            \
    if (!c_) fb_why |= 1u << (bit);              \
  } while (0)
#else
#define NMP_DOM(flag, bit, cond) flag = flag & (((NMP_DOM_MASK >> (bit)) & 1) == 0 || (cond))
#endif
  // ---- vege_flux: func.f90:2465-2964 ----
  T tgv = L(0.0), cmv = L(0.0);
  int vtrips = 0;
  if (veg && fveg > L(0.0)) {
    tgv = c.tg;
    const T mpe = L(1E-6);
    T fv, h, hg, moz, fm, fh, fm2, fh2, fhg, wstar, rahg, rb, rahc, cah, cvh;
    int mozsgn;
    T z0h = z0m;
    T vaie = rmin(L(6.0), vai / fveg);
    T laisune = rmin(L(6.0), laisun / fveg);
    T laishae = rmin(L(6.0), laisha / fveg);
    T tt;
    T estg = esat_val(tdc(tgv));
    T hcan = htop;
    // HCAN = HVT and Z0M = Z0MVT here: LOG(HCAN/Z0M) is veg-type-only
    T uc = ur * ((sizeof(T) == 4 && R) ? (T)V.log_hvt_z0m : M::log(hcan / z0m)) / M::log(zlvl / z0m);
    if ((hcan - zpd) <= L(0.0)) c.status |= NMP_ST_HCAN;
    T air = -emv * (L(1.0) + (L(1.0) - emv) * (L(1.0) - emg)) * c.lwdn -
            emv * emg * SB * p4(tgv);
    T cir = (L(2.0) - emv * (L(1.0) - emg)) * emv * SB;
    T sqrt_dleaf_uc = M::sqrt((T)V.dleaf / uc);  // ragrb :3349, loop-invariant
    const T log_2z0m_v = (T)V.log_2z0m;  // Z0M = Z0MVT: veg-type-only
    Sfc1Logs<T, R> lgv =
        (o.sfc == 1) ? Sfc1Logs<T, R>(zlvl, zpd, z0m, z0h, c.status,
                                      (sizeof(T) == 4 && R) ? &log_2z0m_v : nullptr)
                     : Sfc1Logs<T, R>{};
    // EVC's limit CANLIQ*LATHEAV/DT or CANICE*LATHEAV/DT (:2860-2864): both
    // loop-invariant, the iteration picks one by the canopy temperature
    T evlim_liq = dv(c.canliq * latheav, DT), evlim_ice = dv(c.canice * latheav, DT);
    // The loop-invariant half of the range proof's domain (vege_domain.h,
    // tools/div_proof.py), evaluated once per column before the loop; NaN
    // fails every comparison.
    auto vege_domain_ok = [&]() -> bool {
      auto in = [](T x, double lo, double hi) { return x >= (T)lo && x <= (T)hi; };
      auto zero_or = [&](T x, double lo, double hi) { return x == L(0.0) || in(x, lo, hi); };
      bool k = true;
      NMP_DOM(k, 0, in(c.sfctmp, NMP_DOM_T_LO, NMP_DOM_T_HI) & in(c.tg, NMP_DOM_T_LO, NMP_DOM_T_HI));
      NMP_DOM(k, 1, in(qair, 0.0, 1.0) & in(rhoair, NMP_DOM_RHO_LO, NMP_DOM_RHO_HI));
      NMP_DOM(k, 2, in(c.sfcprs, NMP_DOM_P_LO, NMP_DOM_P_HI) & in(eair, 0.0, NMP_DOM_EAIR_HI));
      NMP_DOM(k, 3, in(ur, 1.0, NMP_DOM_UR_HI));
      NMP_DOM(k, 4, in(lgv.tmpcm, NMP_DOM_TMPC_LO, NMP_DOM_TMPC_HI) &
                        in(lgv.tmpch, NMP_DOM_TMPC_LO, NMP_DOM_TMPC_HI) &
                        in(lgv.tmpcm2, NMP_DOM_TMPC_LO, NMP_DOM_TMPC_HI) &
                        in(lgv.tmpch2, NMP_DOM_TMPC_LO, NMP_DOM_TMPC_HI));
      NMP_DOM(k, 5, in(zlvl - zpd, NMP_DOM_DZ_LO, NMP_DOM_DZ_HI));
      NMP_DOM(k, 6, in(hcan, NMP_DOM_HCAN_LO, NMP_DOM_HCAN_HI) &
                        in(z0m, NMP_DOM_Z0_LO, NMP_DOM_Z0_HI) &
                        in(z0mg, NMP_DOM_Z0_LO, NMP_DOM_Z0_HI) &
                        zero_or(zpd, NMP_DOM_Z0_LO, NMP_DOM_HCAN_HI));
      NMP_DOM(k, 7, (zpd <= hcan) & (z0mg <= hcan) & (z0m + zpd <= L(2.0) * hcan));
      NMP_DOM(k, 8, in(cwp * vaie * hcan, NMP_DOM_CWPH_LO, NMP_DOM_CWPH_HI));
      NMP_DOM(k, 9, in(vaie, NMP_DOM_VAI_LO, 6.0));
      NMP_DOM(k, 10, zero_or(laisune, NMP_DOM_LAI_LO, 6.0) & zero_or(laishae, NMP_DOM_LAI_LO, 6.0));
      NMP_DOM(k, 11, zero_or(c.fwet, NMP_DOM_FWET_LO, 1.0));
      NMP_DOM(k, 12, in(fveg, NMP_DOM_FVEG_LO, 1.0));
      NMP_DOM(k, 13, in(sqrt_dleaf_uc, NMP_DOM_SDL_LO, NMP_DOM_SDL_HI));
      NMP_DOM(k, 14, in(rsurf, 0.0, NMP_DOM_RSURF_HI));
#if NMP_VD_CHECKED & 1
      NMP_DOM(k, 15, in(emg, 0.0, 1.0));  // bounds DTV's denominator A
#endif
#ifdef NMP_VD_NODOMAIN
      k = true;  // (timing probe only: not exact in general)
#endif
      return k;
    };
    // The whole canopy Newton loop (loop1, func.f90:2744-2877) with the
    // division policy `d` (sflx_math.h): every loop variable starts here, so a
    // lane can run it again with the reference's divisions.
    auto vege_loop = [&](auto& d) -> bool {
      constexpr bool kFast = !std::is_same<std::decay_t<decltype(d)>, DivRef<T>>::value;
      // CTR, TR and DTV: their numerators are products of several possibly
      // small factors, outside what the range proof bounds statically
      // (tools/div_proof.py).  IEEE division, or with NMP_VD_CHECKED the
      // loop's policy and a per-lane window on each numerator (`nwin`).
#if defined(NMP_VD_ALLFAST) || (NMP_VD_CHECKED & 1)
      auto& dref = d;  // (NMP_VD_ALLFAST: timing probe only, not exact in general)
#else
      const DivRef<T> dref;
#endif
      // the per-iteration windows of the range proof (vege_domain.h): TV at
      // the start of every iteration, RAHG after every ragrb, RSSUN/RSSHA after
      // the first iteration; any miss sends the lane through the IEEE loop
      bool ok = true;
      auto in = [](T x, T lo, T hi) { return x >= lo && x <= hi; };
      [[maybe_unused]] auto nwin = [](T x) {
        const T ax = fabs(x);
        return (x == L(0.0)) | ((ax >= (T)__builtin_ldexp(1.0, NMP_DOM_NUM_LO_EXP)) &
                                (ax <= (T)__builtin_ldexp(1.0, NMP_DOM_NUM_HI_EXP)));
      };
      cmv = c.cm;
      chv = c.ch;
      fv = L(0.1); h = L(0.0); hg = L(0.0);
      mozsgn = 0;
      moz = fm = fh = fm2 = fh2 = L(0.0);
      fhg = wstar = rahg = rb = cah = cvh = L(0.0);
      rahc = L(1.0);
      c.qsfc = L(0.622) * eair / (c.psfc - L(0.378) * eair);
      int liter = 0;
      // loop-invariant operands of the divisions (same values as the
      // reference forms in every iteration)
      const Sfc1Inv<T> inv = sfc1_inv(d, c.sfctmp, qair, rhoair, zlvl, zpd, z0h);
      const Recip<T> rhcan = d.rec(hcan), rgammav = d.rec(gammav);
      const T dzg = zpd - z0mg, two_vaie = L(2.0) * vaie, fwet_vaie = c.fwet * vaie;
      d.chk(dzg);
      d.chk(two_vaie);
      d.chk(fwet_vaie);
      d.chk(laisune);
      d.chk(laishae);
      // One Newton iteration.  Iteration 1 is peeled (it alone calls
      // stomata/canres, :2779-2803), so the loop that runs the remaining
      // iterations carries none of stomata's code or registers.
      auto vege_iter = [&](const int iter, auto first) -> T {
        if constexpr (!decltype(first)::value) __builtin_assume(iter >= 2);
        if (o.sfc == 1)
          sfcdif1<T, R>(d, inv, iter, h, lgv, ur, mpe, moz, mozsgn, fm, fh, fm2, fh2, cmv, chv, fv,
                        diag_on);
        if (o.sfc == 2) {
          sfcdif2<T, R>(iter, z0m, c.tah, thair, ur, (T)P.g.czil, zlvl, cmv, chv, moz, wstar, fv);
          chv = chv / ur;
          cmv = cmv / ur;
        }
        rahc = rmax(L(1.0), d.divk(L(1.0), d.rec(chv * ur)));
        const Recip<T> rrahc = d.rec(rahc);  // RAWC = RAHC: CAH = CAW, H share it
        ragrb<T, R>(d, inv.rhocp, rhcan, dzg, sqrt_dleaf_uc, iter, vaie, hg, c.tah, zpd, z0mg, hcan,
                    z0h, fv, cwp, mpe, fhg, rahg, rb);
#ifndef NMP_VD_NOWIN
        if constexpr (kFast) NMP_DOM(ok, 16, in(rahg, (T)NMP_DOM_RAHG_LO, (T)NMP_DOM_RAHG_HI));
#endif
        const Recip<T> rrahg = d.rec(rahg), rrb = d.rec(rb);  // RAWG = RAHG
        T estv, destv;
        esat_sel(tdc(c.tv), estv, destv);
        if constexpr (decltype(first)::value) {  // iter == 1
          if (o.crs == 1) {
            const StomataPre<T> sp =
                stomata_pre<T, R>(V, parsun > L(0.0) || parsha > L(0.0), c.sfcprs, c.sfctmp, c.tv,
                                  c.o2air, c.foln, btran, rb);
            // The bisection's divisions: short (DivFast32) in the fast canopy loop
            // when the column and its vegetation type lie in the proven domain
            // (vege_domain.h "stomata", tools/div_proof.py), IEEE otherwise.
            DivRef<T> dsr;
            bool st_fast = false;
            if constexpr (std::is_same_v<std::decay_t<decltype(d)>, DivFast32>) {
              auto in = [](T x, double lo, double hi) { return x >= (T)lo && x <= (T)hi; };
              auto apar_ok = [&](T x) {
                return x <= L(0.0) || in(x, NMP_DOM_APAR_LO, NMP_DOM_APAR_HI);
              };
              st_fast = V.stomata_fast && c.tv <= (T)NMP_DOM_STOMATA_TV_HI &&
                        (c.eah == L(0.0) || in(c.eah, NMP_DOM_EAH_LO, NMP_DOM_EAH_HI)) &&
                        in(c.co2air, NMP_DOM_CO2_LO, NMP_DOM_CO2_HI) &&
                        in(c.o2air, NMP_DOM_O2_LO, NMP_DOM_O2_HI) &&
                        (sp.fnf == L(0.0) || in(sp.fnf, NMP_DOM_FNF_LO, 1.0)) &&
                        apar_ok(parsun) && apar_ok(parsha);
#ifdef NMP_STOMATA_FASTDIV
              st_fast = true;  // (timing probe only: not exact in general)
#endif
#ifdef NMP_COUNT_FALLBACK
              if (!st_fast && (parsun > L(0.0) || parsha > L(0.0)))
                atomicAdd(&nmp_fb_reason[24], 1u);  // stomata bisection on IEEE division
#endif
              if (st_fast) {
                stomata_solve<T, R>(d, V, sp, igs, c.sfcprs, parsun, c.eah, estv, c.co2air,
                                    rssun, psnsun);
                stomata_solve<T, R>(d, V, sp, igs, c.sfcprs, parsha, c.eah, estv, c.co2air,
                                    rssha, psnsha);
              }
            }
            if (!st_fast) {
              stomata_solve<T, R>(dsr, V, sp, igs, c.sfcprs, parsun, c.eah, estv, c.co2air,
                                  rssun, psnsun);
              stomata_solve<T, R>(dsr, V, sp, igs, c.sfcprs, parsha, c.eah, estv, c.co2air,
                                  rssha, psnsha);
            }
          }
          if (o.crs == 2) {
            canres<T, R>(V, c.sfcprs, c.tv, parsun, c.eah, btran, rssun, psnsun);
            canres<T, R>(V, c.sfcprs, c.tv, parsha, c.eah, btran, rssha, psnsha);
          }
#ifndef NMP_VD_NOWIN
          if constexpr (kFast)
            NMP_DOM(ok, 17, in(rssun, L(0.0), (T)NMP_DOM_RS_HI) & in(rssha, L(0.0), (T)NMP_DOM_RS_HI));
#endif
        }
        cah = d.divk(L(1.0), rrahc);
        cvh = d.divk(two_vaie, rrb);
        T cgh = d.divk(L(1.0), rrahg);
        T cond = cah + cvh + cgh;
        const Recip<T> rcond = d.rec(cond);
        T ata = d.div(c.sfctmp * cah + tgv * cgh, rcond);
        T bta = d.div(cvh, rcond);
        T csh = (L(1.0) - bta) * rhoair * CPAIR * cvh;
        T caw = d.divk(L(1.0), rrahc);
        T cew = d.divk(fwet_vaie, rrb);
        T ctw = (L(1.0) - c.fwet) *
                (d.divk(laisune, d.rec(rb + rssun)) + d.divk(laishae, d.rec(rb + rssha)));
        T cgw = d.divk(L(1.0), d.rec(rahg + rsurf));
        cond = caw + cew + ctw + cgw;
        const Recip<T> rcond2 = d.rec(cond);
        T aea = d.div(eair * caw + estg * cgw, rcond2);
        T bea = d.div(cew + ctw, rcond2);
        T cev = d.div((L(1.0) - bea) * cew * rhoair * CPAIR, rgammav);
        const T ctr_n = (L(1.0) - bea) * ctw * rhoair * CPAIR;
#if NMP_VD_CHECKED & 1
        if constexpr (kFast) NMP_DOM(ok, 26, nwin(ctr_n));
#endif
        T ctr = dref.div(ctr_n, rgammav);
        c.tah = ata + bta * c.tv;
        c.eah = aea + bea * estv;
        irc = fveg * (air + cir * p4(c.tv));
        shc = fveg * rhoair * CPAIR * cvh * (c.tv - c.tah);
        evc = d.div(fveg * rhoair * CPAIR * cew * (estv - c.eah), rgammav);
        const T tr_n = fveg * rhoair * CPAIR * ctw * (estv - c.eah);
#if NMP_VD_CHECKED & 1
        if constexpr (kFast) NMP_DOM(ok, 27, nwin(tr_n));
#endif
        tr = dref.div(tr_n, rgammav);
        evc = rmin((c.tv > TFRZ) ? evlim_liq : evlim_ice, evc);
        T b = sav - irc - shc - evc - tr;
        T a = fveg * (L(4.0) * cir * p3(c.tv) + csh + (cev + ctr) * destv);
#if NMP_VD_CHECKED & 1
        if constexpr (kFast) NMP_DOM(ok, 28, nwin(b));
#endif
        T dtv = dref.div(b, dref.rec(a));
        irc = irc + fveg * L(4.0) * cir * p3(c.tv) * dtv;
        shc = shc + fveg * csh * dtv;
        evc = evc + fveg * cev * destv * dtv;
        tr = tr + fveg * ctr * destv * dtv;
        c.tv = c.tv + dtv;
        h = d.div(rhoair * CPAIR * (c.tah - c.sfctmp), rrahc);
        hg = d.div(rhoair * CPAIR * (tgv - c.tah), rrahg);
        c.qsfc = d.div(L(0.622) * c.eah, d.rec(c.sfcprs - L(0.378) * c.eah));
        return dtv;
      };
      if constexpr (kFast) NMP_DOM(ok, 18, in(c.tv, (T)NMP_DOM_T_LO, (T)NMP_DOM_T_HI));
      vtrips = 1;
      vege_iter(1, std::true_type{});  // iter 1 cannot exit (the test needs iter >= 5)
      NMP_UNROLL(NMP_VEGE_UNROLL)
      for (int iter = 2; iter <= 20; ++iter) {
        vtrips = iter;
        if constexpr (kFast) NMP_DOM(ok, 19, in(c.tv, (T)NMP_DOM_T_LO, (T)NMP_DOM_TV_HI));
        const T dtv = vege_iter(iter, std::false_type{});
        if (liter == 1) break;
        if (iter >= 5 && fabs(dtv) <= L(0.01) && liter == 0) liter = 1;
      }
      return ok;
    };
    DivRef<T> dr;
#if NMP_VEGE_DIV
    if constexpr (sizeof(T) == 4 && R && OS != 0) {
      // the short exact division wherever the range proofs hold; a lane
      // outside their window repeats the loop from its start with IEEE
      // division (TV/TAH/EAH reloaded: nothing has stored them yet)
      DivFast32 df;
#ifdef NMP_VD_NOFALLBACK
      (void)vege_domain_ok();
      vege_loop(df);
      if (false) {  // (timing probe only: not exact in general)
#else
      if (!vege_domain_ok() || !vege_loop(df)) {
#endif
#ifdef NMP_COUNT_FALLBACK
        atomicAdd(&nmp_fallback_ctr, 1u);
        for (int b = 0; b < 29; ++b)
          if ((0x1c0fffffu >> b) & (fb_why >> b) & 1u) atomicAdd(&nmp_fb_reason[b], 1u);
#endif
        c.tv = out.ls(NMP_S_TV);
        c.tah = out.ls(NMP_S_TAH);
        c.eah = out.ls(NMP_S_EAH);
        vege_loop(dr);
      }
    } else {
      vege_loop(dr);
    }
#else
    vege_loop(dr);
#endif
    // under-canopy fluxes and TG (loop2, :2881-2914)
    air = -emg * (L(1.0) - emv) * c.lwdn - emg * emv * SB * p4(c.tv);
    cir = emg * SB;
    T csh = rhoair * CPAIR / rahg;
    T cev = rhoair * CPAIR / (gammag * (rahg + rsurf));
    T cgh = L(2.0) * df_top / dz_top;
NMP_UNROLL(NMP_LOOP2_UNROLL)
    for (int iter = 1; iter <= 5; ++iter) {
      tt = tdc(tgv);
      T destg;
      esat_sel(tt, estg, destg);
      irg = cir * p4(tgv) + air;
      shg = csh * (tgv - c.tah);
      evg = cev * (estg * rhsur - c.eah);
      ghv = cgh * (tgv - stc_top);
      T b = sag - irg - shg - evg - ghv;
      T a = L(4.0) * cir * p3(tgv) + csh + cev * destg + cgh;
      T dtg = dv(b, a);
      irg = irg + L(4.0) * cir * p3(tgv) * dtg;
      shg = shg + csh * dtg;
      evg = evg + cev * destg * dtg;
      ghv = ghv + cgh * dtg;
      tgv = tgv + dtg;
    }
    if (o.stc == 1 && c.snowh > L(0.05) && tgv > TFRZ) {
      tgv = TFRZ;
      irg = cir * p4(tgv) - emg * (L(1.0) - emv) * c.lwdn - emg * emv * SB * p4(c.tv);
      shg = csh * (tgv - c.tah);
      evg = cev * (estg * rhsur - c.eah);
      ghv = sag - (irg + shg + evg);
    }
    if ((o.sfc == 1 || o.sfc == 2) && diag_on) {
      chv2 = fv * KARMAN / (((o.sfc == 1) ? lgv.tmpch2 : M::log((L(2.0) + z0h) / z0h)) - fh2);
      if (chv2 < L(1.E-5)) {
        t2mv = c.tah;
        q2v = c.qsfc;
      } else {
        t2mv = c.tah - (shg + shc / fveg) / (rhoair * CPAIR) * L(1.0) / chv2;
        q2v = c.qsfc - ((evc + tr) / fveg + evg) / (latheav * rhoair) * L(1.0) / chv2;
      }
    }
    chv = cah;
    chleaf = cvh;
    chuc = L(1.0) / rahg;
  }
  out.trips(vtrips);

  NMP_PHASE(5);
  // ---- bare_flux: func.f90:2967-3257 ----
  T tgb = c.tg, cmb = c.cm, chb = c.ch;
  T irb, shb, evb, ghb, t2mb = L(0.0), q2b = L(0.0), chb2 = L(0.0);
  {
    const T mpe = L(1.0E-6);
    int mozsgn;
    T h, fv, moz, fm, fh, fm2, fh2, wstar;
    T cir = emg * SB;
    T cgh = L(2.0) * df_top / dz_top;
    T z0h = z0mg, ehb, csh, cev, estg;
    // saturation pressure at TGB: each iteration's closing value is the next
    // iteration's opening value (same TGB), so it is carried, not recomputed
    T es_tgb, des_tgb;
    const Sfc1Logs<T, R> lgb = (o.sfc == 1) ? Sfc1Logs<T, R>(zlvl, zpdg, z0mg, z0h, c.status)
                                            : Sfc1Logs<T, R>{};
    // The bare-ground Newton loop (func.f90:3120-3200) with the division
    // policy `d`, as the canopy loop: every loop variable starts here, so a
    // lane outside the range proof's domain can run it again with IEEE
    // division.  DTG = B/A: IEEE division, or with NMP_VD_CHECKED & 2 the
    // loop's policy and a per-lane window on B.
    auto bare_loop = [&](auto& d) -> bool {
      constexpr bool kFast = !std::is_same<std::decay_t<decltype(d)>, DivRef<T>>::value;
#if NMP_VD_CHECKED & 2
      auto& dref = d;
#else
      const DivRef<T> dref;
#endif
      bool ok = true;
      auto in = [](T x, T lo, T hi) { return x >= lo && x <= hi; };
      [[maybe_unused]] auto nwin = [](T x) {
        const T ax = fabs(x);
        return (x == L(0.0)) | ((ax >= (T)__builtin_ldexp(1.0, NMP_DOM_NUM_LO_EXP)) &
                                (ax <= (T)__builtin_ldexp(1.0, NMP_DOM_NUM_HI_EXP)));
      };
      tgb = c.tg;
      cmb = c.cm;
      chb = c.ch;
      mozsgn = 0;
      h = L(0.0); fv = L(0.1); moz = L(0.0); fm = L(0.0); fh = L(0.0); fm2 = L(0.0); fh2 = L(0.0);
      wstar = L(0.0);
      ehb = csh = cev = estg = L(0.0);
      esat_sel(tdc(tgb), es_tgb, des_tgb);
      irb = shb = evb = ghb = L(0.0);
      const Sfc1Inv<T> invb = sfc1_inv(d, c.sfctmp, qair, rhoair, zlvl, zpdg, z0h);
NMP_UNROLL(NMP_BARE_UNROLL)
      for (int iter = 1; iter <= 5; ++iter) {
        if constexpr (kFast) NMP_DOM(ok, 20, in(tgb, (T)NMP_DOM_T_LO, (T)NMP_DOM_TGB_HI));
        if (o.sfc == 1)
          sfcdif1<T, R>(d, invb, iter, h, lgb, ur, mpe, moz, mozsgn, fm, fh, fm2, fh2, cmb, chb, fv,
                        diag_on);
        if (o.sfc == 2) {
          sfcdif2<T, R>(iter, z0mg, tgb, thair, ur, (T)P.g.czil, zlvl, cmb, chb, moz, wstar, fv);
          chb = chb / ur;
          cmb = cmb / ur;
          if (c.snowh > L(0.0)) {
            cmb = rmin(L(0.01), cmb);
            chb = rmin(L(0.01), chb);
          }
        }
        T rahb = rmax(L(1.0), d.divk(L(1.0), d.rec(chb * ur)));
        const Recip<T> rrahb = d.rec(rahb);  // RAWB = RAHB
        ehb = d.divk(L(1.0), rrahb);
        estg = es_tgb;
        const T destg = des_tgb;
        csh = d.div(rhoair * CPAIR, rrahb);
        cev = d.div(d.div(rhoair * CPAIR, d.rec(gammag)), d.rec(rsurf + rahb));
        irb = cir * p4(tgb) - emg * c.lwdn;
        shb = csh * (tgb - c.sfctmp);
        evb = cev * (estg * rhsur - eair);
        ghb = cgh * (tgb - stc_top);
        T b = sag - irb - shb - evb - ghb;
        T a = L(4.0) * cir * p3(tgb) + csh + cev * destg + cgh;
#if NMP_VD_CHECKED & 2
        if constexpr (kFast) NMP_DOM(ok, 29, nwin(b));
#endif
        T dtg = dref.div(b, dref.rec(a));
        irb = irb + L(4.0) * cir * p3(tgb) * dtg;
        shb = shb + csh * dtg;
        evb = evb + cev * destg * dtg;
        ghb = ghb + cgh * dtg;
        tgb = tgb + dtg;
        h = csh * (tgb - c.sfctmp);
        esat_sel(tdc(tgb), es_tgb, des_tgb);
        estg = es_tgb;
        // QSFC is overwritten every iteration and read only after the loop
        if (iter == 5) c.qsfc = L(0.622) * (estg * rhsur) / (c.psfc - L(0.378) * (estg * rhsur));
      }
      return ok;
    };
    // the loop-invariant half of the bare loop's domain (vege_domain.h)
    auto bare_domain_ok = [&]() -> bool {
      auto in = [](T x, double lo, double hi) { return x >= (T)lo && x <= (T)hi; };
      bool k = true;
      NMP_DOM(k, 21, in(c.sfctmp, NMP_DOM_T_LO, NMP_DOM_T_HI) & in(qair, 0.0, 1.0) &
                         in(rhoair, NMP_DOM_RHO_LO, NMP_DOM_RHO_HI) &
                         in(c.sfcprs, NMP_DOM_P_LO, NMP_DOM_P_HI) & in(ur, 1.0, NMP_DOM_UR_HI));
      NMP_DOM(k, 22, in(lgb.tmpcm, NMP_DOM_TMPC_LO, NMP_DOM_TMPC_HI) &
                         in(lgb.tmpch, NMP_DOM_TMPC_LO, NMP_DOM_TMPC_HI) &
                         in(lgb.tmpcm2, NMP_DOM_TMPC_LO, NMP_DOM_TMPC_HI) &
                         in(lgb.tmpch2, NMP_DOM_TMPC_LO, NMP_DOM_TMPC_HI));
      NMP_DOM(k, 23, in(zlvl - zpdg, NMP_DOM_DZ_LO, NMP_DOM_DZ_HI) &
                         in(z0mg, NMP_DOM_Z0_LO, NMP_DOM_Z0_HI) & in(rsurf, 0.0, NMP_DOM_RSURF_HI));
#if NMP_VD_CHECKED & 2
      NMP_DOM(k, 30, in(emg, 0.0, 1.0) & in(cgh, 0.0, NMP_DOM_CGH_HI));  // DTG's A
#endif
#ifdef NMP_VD_NODOMAIN
      k = true;
#endif
      return k;
    };
    DivRef<T> drb;
#if NMP_VEGE_DIV && NMP_BARE_DIV
    if constexpr (sizeof(T) == 4 && R && OS != 0) {
      DivFast32 dfb;
      if (!bare_domain_ok() || !bare_loop(dfb)) {
#ifdef NMP_COUNT_FALLBACK
        atomicAdd(&nmp_fallback_ctr, 1u);
        for (int b = 20; b < 31; ++b)
          if ((0x60f00000u >> b) & (fb_why >> b) & 1u) atomicAdd(&nmp_fb_reason[b], 1u);
#endif
        bare_loop(drb);
      }
    } else {
      bare_loop(drb);
    }
#else
    bare_loop(drb);
#endif
    if (o.stc == 1 && c.snowh > L(0.05) && tgb > TFRZ) {
      tgb = TFRZ;
      irb = cir * p4(tgb) - emg * c.lwdn;
      shb = csh * (tgb - c.sfctmp);
      evb = cev * (estg * rhsur - eair);
      ghb = sag - (irb + shb + evb);
    }
    if ((o.sfc == 1 || o.sfc == 2) && diag_on) {
      chb2 = fv * KARMAN / (((o.sfc == 1) ? lgb.tmpch2 : M::log((L(2.0) + z0h) / z0h)) - fh2);
      if (chb2 < L(1.0E-5)) {
        t2mb = tgb;
        q2b = c.qsfc;
      } else {
        t2mb = tgb - shb / (rhoair * CPAIR) * L(1.0) / chb2;
        q2b = c.qsfc - evb / (latheag * rhoair) * (L(1.0) / chb2 + rsurf);
      }
      if (c.lutyp == P.g.isurban) q2b = c.qsfc;
    }
    chb = ehb;
  }

#if NMP_EARLY_LOADS & 1
  // the water phase's fields issued here, their latency under aggregation,
  // thermoprop, tsnosoi and phasechange
  NMP_WATER_LOADS();
#endif
  NMP_PHASE(6);
  // tile aggregation (:1246-1282)
  T fira, fsh, fgev, ssoil, fcev, fctr, t2m;
  if (veg && fveg > L(0.0)) {
    fira = fveg * irg + (L(1.0) - fveg) * irb + irc;
    fsh = fveg * shg + (L(1.0) - fveg) * shb + shc;
    fgev = fveg * evg + (L(1.0) - fveg) * evb;
    ssoil = fveg * ghv + (L(1.0) - fveg) * ghb;
    fcev = evc;
    fctr = tr;
    c.tg = fveg * tgv + (L(1.0) - fveg) * tgb;
    t2m = fveg * t2mv + (L(1.0) - fveg) * t2mb;
    c.cm = fveg * cmv + (L(1.0) - fveg) * cmb;
    c.ch = fveg * chv + (L(1.0) - fveg) * chb;
  } else {
    fira = irb;
    fsh = shb;
    fgev = evb;
    ssoil = ghb;
    c.tg = tgb;
    t2m = t2mb;
    fcev = L(0.);
    fctr = L(0.);
    c.cm = cmb;
    c.ch = chb;
    rssun = L(0.0);
    rssha = L(0.0);
    tgv = tgb;
    chv = chb;
  }
  T fire = c.lwdn + fira;
  if (fire <= L(0.0)) c.status |= NMP_ST_FIRE;
  T emissi = fveg * (emg * (L(1.) - emv) + emv + emv * (L(1.) - emv) * (L(1.) - emg)) +
             (L(1.) - fveg) * emg;
  T trad = diag_on ? M::pow_q((fire - (L(1.0) - emissi) * c.lwdn) / (emissi * SB)) : L(0.0);
  T apar = parsun * laisun + parsha * laisha;
  T psn = psnsun * laisun + psnsha * laisha;
  // error(): energy balance (func.f90:712-721), a function of final energy terms only
  if (fabs(sav + sag - (fira + fsh + fcev + fgev + fctr + ssoil)) > L(0.01))
    c.status |= NMP_ST_ERRENG;
  out.template d<NMP_D_SAV>(sav);
  out.template d<NMP_D_SAG>(sag);
  out.template d<NMP_D_FIRA>(fira);
  out.template d<NMP_D_SSOIL>(ssoil);
  out.template d<NMP_D_FSH>(fsh);
  out.template d<NMP_D_FCEV>(fcev);
  out.template d<NMP_D_FGEV>(fgev);
  out.template d<NMP_D_FCTR>(fctr);
  out.template d<NMP_D_TRAD>(trad);
  out.template d<NMP_D_T2MV>(t2mv);
  out.template d<NMP_D_T2MB>(t2mb);
  out.template d<NMP_D_Q2V>(q2v);
  out.template d<NMP_D_APAR>(apar);
  out.template d<NMP_D_PSN>(psn);
  out.template d<NMP_D_RSSUN>(rssun);
  out.template d<NMP_D_RSSHA>(rssha);
  out.template d<NMP_D_CHV>(chv);
  out.template d<NMP_D_CHB>(chb);
  out.template d<NMP_D_EMISSI>(emissi);
  out.template d<NMP_D_SHG>(shg);
  out.template d<NMP_D_SHC>(shc);
  out.template d<NMP_D_SHB>(shb);
  out.template d<NMP_D_EVG>(evg);
  out.template d<NMP_D_EVB>(evb);
  out.template d<NMP_D_GHV>(ghv);
  out.template d<NMP_D_GHB>(ghb);
  out.template d<NMP_D_IRG>(irg);
  out.template d<NMP_D_IRC>(irc);
  out.template d<NMP_D_IRB>(irb);
  out.template d<NMP_D_TR>(tr);
  out.template d<NMP_D_EVC>(evc);
  out.template d<NMP_D_CHLEAF>(chleaf);
  out.template d<NMP_D_CHUC>(chuc);
  out.template d<NMP_D_CHV2>(chv2);
  out.template d<NMP_D_CHB2>(chb2);
  out.t2m(t2m);
  out.s(NMP_S_TAH, c.tah);
  out.s(NMP_S_EAH, c.eah);
  out.s(NMP_S_CM, c.cm);
  out.s(NMP_S_CH, c.ch);

  // Re-read the layer state (unchanged in HBM so far) instead of holding it in
  // registers through the flux iterations; then FICEOLD and thermoprop.
  {
    // from the LDS copy (kPrefetch) or from HBM
    const T* st = out.fresh_state();
    // the LDS slot index is laundered like fresh_state(): a real second read,
    // not the entry values kept live in registers through the flux loops
    int slot = threadIdx.x;
    if constexpr (kPfReread<T, R>) __asm__ volatile("" : "+v"(slot));
    auto rd = [&](int f) -> T {
      if constexpr (kPfReread<T, R>)
        return lds_pool()[f * NMP_BLOCK + slot];
      else
        return gld(col_at(st, out.ld, out.col, f));
    };
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      c.stc[k] = rd(NMP_S_STC + k);
      c.zsnso[k] = rd(NMP_S_ZSNSO + k);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      c.snice[k] = rd(NMP_S_SNICE + k);
      c.snliq[k] = rd(NMP_S_SNLIQ + k);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c.sh2o[k] = rd(NMP_S_SH2O + k);
      c.smc[k] = rd(NMP_S_SMC + k);
    }
    layer_dz(c);
  }
  // FICEOLD: the caller's (nmp_sflx_columns, noahmp_sflx's intent(in) argument)
  // or, by default, the state's ice fraction at step start (offline-driver
  // convention)
  if (out.fice) {
#pragma unroll
    for (int j = 0; j < 3; ++j) c.ficeold[j] = *out.at(out.fice, j);
  } else {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      c.ficeold[j] = (j >= c.isnow + 3) ? c.snice[j] / (c.snice[j] + c.snliq[j]) : L(0.0);
  }
  NMP_PHASE(14);
  // thermoprop + csnow + tdfcnd: func.f90:1341-1595
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j >= kt) {
      T snicev = rmin(L(1.0), c.snice[j] / (c.dz[j] * DENICE));
      T epore = L(1.0) - snicev;
      T snliqv = rmin(epore, c.snliq[j] / (c.dz[j] * DENWAT));
      T bdsnoi = (c.snice[j] + c.snliq[j]) / c.dz[j];
      c.hcpct[j] = CICE * snicev + CWAT * snliqv;
      c.df[j] = L(3.2217E-6) * p2(bdsnoi);
    } else {
      c.hcpct[j] = L(0.0);
      c.df[j] = L(0.0);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    T sice = c.smc[k] - c.sh2o[k];
    c.hcpct[k + 3] = c.sh2o[k] * CWAT + (L(1.0) - smcmax) * (T)P.g.csoil +
                     (smcmax - c.smc[k]) * CPAIR + sice * CICE;
    c.df[k + 3] = tdfcnd<T, R>(S, c.smc[k], c.sh2o[k]);
  }
  if (c.lutyp == P.g.isurban) {
#pragma unroll
    for (int k = 3; k < 7; ++k) c.df[k] = L(3.24);
  }
  if (c.ist == 2) {
#pragma unroll
    for (int k = 3; k < 7; ++k) {
      const bool warm = c.stc[k] > TFRZ;
      c.hcpct[k] = warm ? CWAT : CICE;
      c.df[k] = warm ? TKWAT : TKICE;
    }
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) c.fact[k] = (k >= kt) ? DT / (c.hcpct[k] * c.dz[k]) : L(0.0);
  if (c.isnow == 0)
    c.df[3] = (c.df[3] * c.dz[3] + L(0.35) * c.snowh) / (c.snowh + c.dz[3]);
  else
    c.df[3] = (c.df[3] * c.dz[3] + c.df[2] * c.dz[2]) / (c.dz[2] + c.dz[3]);

  NMP_PHASE(7);
  // tsnosoi + hrt + hstep (func.f90:3987-4237), layers kt..6 in VGPRs
  {
    T ai[7], bi[7], ci[7], rhs[7], ddz[7], denom[7], dtsdz[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) ai[k] = bi[k] = ci[k] = rhs[k] = ddz[k] = denom[k] = dtsdz[k] = L(0.);
    const T zbotsno = (T)P.g.zbot - c.snowh;
    T botflx = L(0.0);
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int km = k > 0 ? k - 1 : 0, kp = k < 6 ? k + 1 : 6;
      if (k == kt) {
        denom[k] = -c.zsnso[k] * c.hcpct[k];
        T temp1 = -c.zsnso[kp];
        ddz[k] = L(2.0) / temp1;
        dtsdz[k] = L(2.0) * (c.stc[k] - c.stc[kp]) / temp1;
        rhs[k] = c.df[k] * dtsdz[k] - ssoil - L(0.0);  // EFLUX
      } else if (k > kt && k < 6) {
        denom[k] = (c.zsnso[km] - c.zsnso[k]) * c.hcpct[k];
        T temp1 = c.zsnso[km] - c.zsnso[kp];
        ddz[k] = L(2.0) / temp1;
        dtsdz[k] = L(2.0) * (c.stc[k] - c.stc[kp]) / temp1;
        rhs[k] = (c.df[k] * dtsdz[k] - c.df[km] * dtsdz[km]) - L(0.0);
      } else if (k == 6) {
        denom[k] = (c.zsnso[km] - c.zsnso[k]) * c.hcpct[k];
        if (o.tbot == 1) botflx = L(0.);
        if (o.tbot == 2) {
          dtsdz[k] = (c.stc[k] - c.tbot) / (L(0.5) * (c.zsnso[km] + c.zsnso[k]) - zbotsno);
          botflx = -c.df[k] * dtsdz[k];
        }
        rhs[k] = (-botflx - c.df[km] * dtsdz[km]) - L(0.0);
      }
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int km = k > 0 ? k - 1 : 0;
      if (k == kt) {
        ai[k] = L(0.0);
        ci[k] = -c.df[k] * ddz[k] / denom[k];
        if (o.stc == 1) bi[k] = -ci[k];
        if (o.stc == 2) bi[k] = -ci[k] + c.df[k] / (L(0.5) * c.zsnso[k] * c.zsnso[k] * c.hcpct[k]);
      } else if (k > kt && k < 6) {
        ai[k] = -c.df[km] * ddz[km] / denom[k];
        ci[k] = -c.df[k] * ddz[k] / denom[k];
        bi[k] = -(ai[k] + ci[k]);
      } else if (k == 6) {
        ai[k] = -c.df[km] * ddz[km] / denom[k];
        ci[k] = L(0.0);
        bi[k] = -(ai[k] + ci[k]);
      }
      if (k >= kt) rhs[k] = rhs[k] / (-denom[k]);
    }
    T ciin[7], rhsin[7], pp[7], delta[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      if (k >= kt) {
        rhs[k] = rhs[k] * DT;
        ai[k] = ai[k] * DT;
        bi[k] = L(1.) + bi[k] * DT;
        ci[k] = ci[k] * DT;
      }
      rhsin[k] = rhs[k];
      ciin[k] = ci[k];
      pp[k] = L(0.);
      delta[k] = L(0.);
    }
    rosr12<T, 7>(pp, ai, bi, ciin, rhsin, delta, kt);
#pragma unroll
    for (int k = 0; k < 7; ++k)
      if (k >= kt) c.stc[k] = c.stc[k] + pp[k];
  }
  if (o.stc == 2) {
    if (c.snowh > L(0.05) && c.tg > TFRZ) {
      tgv = TFRZ;
      tgb = TFRZ;
      c.tg = (veg && fveg > L(0.0)) ? fveg * tgv + (L(1.0) - fveg) * tgb : tgb;
    }
  }
  out.template d<NMP_D_TGB>(tgb);
  out.template d<NMP_D_TGV>(tgv);
  out.s(NMP_S_TG, c.tg);

  NMP_PHASE(8);
  // phasechange: func.f90:4291-4491
  T qmelt = L(0.0), ponding = L(0.0);
  {
    T hm[7], xm[7], wmass0[7], wice0[7], mice[7], mliq[7], supercool[7];
    T xmf = L(0.0);
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      supercool[k] = L(0.0);
      if (k < 3) {
        mice[k] = c.snice[k];
        mliq[k] = c.snliq[k];
      } else {
        mliq[k] = c.sh2o[k - 3] * c.dz[k] * L(1000.0);
        mice[k] = (c.smc[k - 3] - c.sh2o[k - 3]) * c.dz[k] * L(1000.0);
      }
      c.imelt[k] = 0;
      hm[k] = L(0.0);
      xm[k] = L(0.0);
      wice0[k] = mice[k];
      wmass0[k] = mice[k] + mliq[k];
    }
    if (c.ist == 1) {
#pragma unroll
      for (int k = 3; k < 7; ++k) {
        if (o.frz == 1 && c.stc[k] < TFRZ) {
          T smp = HFUS * (TFRZ - c.stc[k]) / (GRAV * c.stc[k]);
          supercool[k] = smcmax * M::pow(smp / psisat, L(-1.0) / bexp);
          supercool[k] = supercool[k] * c.dz[k] * L(1000.0);
        }
        if (o.frz == 2) {  // frh2o: func.f90:4494-4598 (sflx_routines.h)
          const T free_ = frh2o<T, R>(smcmax, psisat, bexp, c.stc[k], c.smc[k - 3],
                                      c.sh2o[k - 3], c.status);
          supercool[k] = free_ * c.dz[k] * L(1000.0);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      if (k >= kt) {
        if (mice[k] > L(0.0) && c.stc[k] >= TFRZ) c.imelt[k] = 1;
        if (mliq[k] > supercool[k] && c.stc[k] < TFRZ) c.imelt[k] = 2;
        if (k == 3 && c.isnow == 0 && c.sneqv > L(0.0) && c.stc[k] >= TFRZ) c.imelt[k] = 1;
      }
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      if (k >= kt) {
        if (c.imelt[k] > 0) {
          hm[k] = (c.stc[k] - TFRZ) / c.fact[k];
          c.stc[k] = TFRZ;
        }
        if (c.imelt[k] == 1 && hm[k] < L(0.0)) {
          hm[k] = L(0.0);
          c.imelt[k] = 0;
        }
        if (c.imelt[k] == 2 && hm[k] > L(0.0)) {
          hm[k] = L(0.0);
          c.imelt[k] = 0;
        }
        xm[k] = hm[k] * DT / HFUS;
      }
    }
    if (c.isnow == 0 && c.sneqv > L(0.0) && xm[3] > L(0.0)) {
      T temp1 = c.sneqv;
      c.sneqv = rmax(L(0.0), temp1 - xm[3]);
      T propor = c.sneqv / temp1;
      c.snowh = rmax(L(0.0), propor * c.snowh);
      T heatr = hm[3] - HFUS * (temp1 - c.sneqv) / DT;
      if (heatr > L(0.0)) {
        xm[3] = heatr * DT / HFUS;
        hm[3] = heatr;
      } else {
        xm[3] = L(0.0);
        hm[3] = L(0.0);
      }
      qmelt = rmax(L(0.0), (temp1 - c.sneqv)) / DT;
      xmf = HFUS * qmelt;
      ponding = temp1 - c.sneqv;
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      if (k >= kt && c.imelt[k] > 0 && fabs(hm[k]) > L(0.0)) {
        T heatr = L(0.0);
        if (xm[k] > L(0.0)) {
          mice[k] = rmax(L(0.0), wice0[k] - xm[k]);
          heatr = hm[k] - HFUS * (wice0[k] - mice[k]) / DT;
        } else if (xm[k] < L(0.0)) {
          if (k < 3) {
            mice[k] = rmin(wmass0[k], wice0[k] - xm[k]);
          } else {
            if (wmass0[k] < supercool[k]) {
              mice[k] = L(0.0);
            } else {
              mice[k] = rmin(wmass0[k] - supercool[k], wice0[k] - xm[k]);
              mice[k] = rmax(mice[k], L(0.0));
            }
          }
          heatr = hm[k] - HFUS * (wice0[k] - mice[k]) / DT;
        }
        mliq[k] = rmax(L(0.0), wmass0[k] - mice[k]);
        if (fabs(heatr) > L(0.0)) {
          c.stc[k] = c.stc[k] + c.fact[k] * heatr;
          if (k < 3 && mliq[k] * mice[k] > L(0.0)) c.stc[k] = TFRZ;
        }
        xmf = xmf + HFUS * (wice0[k] - mice[k]) / DT;
        if (k < 3) qmelt = qmelt + rmax(L(0.0), (wice0[k] - mice[k])) / DT;
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k >= kt) {
        c.snliq[k] = mliq[k];
        c.snice[k] = mice[k];
      }
    }
#pragma unroll
    for (int k = 3; k < 7; ++k) {
      c.sh2o[k - 3] = mliq[k] / (L(1000.0) * c.dz[k]);
      c.smc[k - 3] = (mliq[k] + mice[k]) / (L(1000.0) * c.dz[k]);
    }
    (void)xmf;
  }
  // ===================== end energy =====================
  out.template d<NMP_D_PONDING>(ponding);

#pragma unroll
  for (int k = 0; k < 4; ++k) c.sice[k] = rmax(L(0.0), c.smc[k] - c.sh2o[k]);
  c.sneqvo = c.sneqv;
  const T qvap = rmax(fgev / latheag, L(0.0));
  const T qdew = fabs(rmin(fgev / latheag, L(0.0)));
  const T edir = qvap - qdew;
  out.template d<NMP_D_EDIR>(edir);
  out.s(NMP_S_SNEQVO, c.sneqvo);
#ifdef NMP_TRUNC_ENERGY
  return;  // timing experiment only (tools/build_variants.py): the energy phase alone
#endif

  NMP_PHASE(9);
  // ===================== water: func.f90:4601-4804 =====================
  // fields first used by the water / carbon phase
#if !(NMP_EARLY_LOADS & 1)
  NMP_WATER_LOADS();
#endif
  const T qprecc = L(0.10) * prcp_w;  // atm :517-518
  const T qprecl = L(0.90) * prcp_w;
  T ecan, etran, runsrf = L(0.0), runsub = L(0.0), qsnbot = L(0.0), ponding1 = L(0.0);
  T ponding2 = L(0.0), fpice = L(0.0), snoflow = L(0.0);
  T qrain, snowhin;
  {
    // canwater: func.f90:4807-5046
    T fp = L(0.0), qintr, qdripr, qthror, qints, qdrips, qthros, qevac, qdewc, qfroc, qsubc;
    if (o.snf == 1) {
      if (c.sfctmp > TFRZ + L(2.5))
        fpice = L(0.0);
      else if (c.sfctmp <= TFRZ + L(0.5))
        fpice = L(1.0);
      else if (c.sfctmp <= TFRZ + L(2.0))
        fpice = L(1.0) - (L(-54.632) + L(0.2) * c.sfctmp);
      else
        fpice = L(0.6);
    }
    if (o.snf == 2) fpice = (c.sfctmp >= TFRZ + L(2.2)) ? L(0.) : L(1.0);
    if (o.snf == 3) fpice = (c.sfctmp >= TFRZ) ? L(0.0) : L(1.0);
    T bdfall = rmin(L(120.0), L(67.92) + L(51.25) * M::exp((c.sfctmp - TFRZ) / L(2.59)));
    T rain = (qprecc + qprecl) * (L(1.0) - fpice);
    T snow = (qprecc + qprecl) * fpice;
    if (qprecc + qprecl > L(0.0)) fp = (qprecc + qprecl) / (L(10.0) * qprecc + qprecl);
    T maxliq = (T)V.canwmxp * (elai + esai);
    if ((elai + esai) > L(0.0)) {
      qintr = fveg * rain * fp;
      // no rain: EXP(-0) = 1 makes the bound +-0 (or NaN), and QINTR ends +0
      // through the MAX below either way, so the exponential is skipped
      if (rain != L(0.0))
        qintr = rmin(qintr, (maxliq - c.canliq) / DT * (L(1.0) - M::exp(-rain * DT / maxliq)));
      qintr = rmax(qintr, L(0.0));
      qdripr = fveg * rain - qintr;
      qthror = (L(1.0) - fveg) * rain;
    } else {
      qintr = L(0.0);
      qdripr = L(0.0);
      qthror = rain;
    }
    if (!frozen_canopy) {
      etran = rmax(fctr / HVAP, L(0.0));
      qevac = rmax(fcev / HVAP, L(0.0));
      qdewc = fabs(rmin(fcev / HVAP, L(0.0)));
      qsubc = L(0.0);
      qfroc = L(0.0);
    } else {
      etran = rmax(fctr / HSUB, L(0.0));
      qevac = L(0.0);
      qdewc = L(0.0);
      qsubc = rmax(fcev / HSUB, L(0.0));
      qfroc = fabs(rmin(fcev / HSUB, L(0.0)));
    }
    qevac = rmin(c.canliq / DT, qevac);
    c.canliq = rmax(L(0.0), c.canliq + (qintr + qdewc - qevac) * DT);
    if (c.canliq <= L(1.0E-6)) c.canliq = L(0.0);
    T maxsno = L(6.6) * (L(0.27) + L(46.0) / bdfall) * (elai + esai);
    if ((elai + esai) > L(0.0)) {
      qints = fveg * snow * fp;
      if (snow != L(0.0))  // as QINTR: no snow leaves QINTS = +0
        qints = rmin(qints, (maxsno - c.canice) / DT * (L(1.0) - M::exp(-snow * DT / maxsno)));
      qints = rmax(qints, L(0.0));
      T ft = rmax(L(0.0), (c.tv - L(270.15)) / L(1.87E5));
      T fvw = M::sqrt(uu_w * uu_w + vv_w * vv_w) / L(1.56E5);
      qdrips = rmax(L(0.0), c.canice) * (fvw + ft);
      qthros = (L(1.0) - fveg) * snow + (fveg * snow - qints);
    } else {
      qints = L(0.0);
      qdrips = L(0.0);
      qthros = snow;
    }
    qsubc = rmin(c.canice / DT, qsubc);
    c.canice = rmax(L(0.0), c.canice + (qints - qdrips) * DT + (qfroc - qsubc) * DT);
    if (c.canice <= L(1.0E-6)) c.canice = L(0.0);
    if (c.canice > L(0.0))
      c.fwet = rmax(L(0.0), c.canice) / rmax(maxsno, L(1.0E-06));
    else
      c.fwet = rmax(L(0.0), c.canliq) / rmax(maxliq, L(1.0E-06));
    c.fwet = M::pow(rmin(c.fwet, L(1.0)), L(0.667));
    if (c.canice > L(1.0E-6) && c.tv > TFRZ) {
      T qmeltc = rmin(c.canice / DT, (c.tv - TFRZ) * CICE * c.canice / DENICE / (DT * HFUS));
      c.canice = rmax(L(0.0), c.canice - qmeltc * DT);
      c.canliq = rmax(L(0.0), c.canliq + qmeltc * DT);
      c.tv = c.fwet * TFRZ + (L(1.0) - c.fwet) * c.tv;
    }
    if (c.canliq > L(1.0E-6) && c.tv < TFRZ) {
      T qfrzc = rmin(c.canliq / DT, (TFRZ - c.tv) * CWAT * c.canliq / DENWAT / (DT * HFUS));
      c.canliq = rmax(L(0.0), c.canliq - qfrzc * DT);
      c.canice = rmax(L(0.0), c.canice + qfrzc * DT);
      c.tv = c.fwet * TFRZ + (L(1.0) - c.fwet) * c.tv;
    }
    ecan = qevac + qsubc - qdewc - qfroc;
    qrain = qdripr + qthror;
    c.qsnow = qdrips + qthros;
    snowhin = c.qsnow / bdfall;
    if (c.ist == 2 && c.tg > TFRZ) {
      c.qsnow = L(0.0);
      snowhin = L(0.0);
    }
  }
  // canopy water / temperature are final after canwater
  out.s(NMP_S_CANLIQ, c.canliq); out.s(NMP_S_CANICE, c.canice);
  out.s(NMP_S_FWET, c.fwet); out.s(NMP_S_TV, c.tv); out.s(NMP_S_QSNOW, c.qsnow);
  out.template d<NMP_D_ECAN>(ecan);
  out.template d<NMP_D_ETRAN>(etran);
  out.template d<NMP_D_FPICE>(fpice);
  T qsnsub = (c.sneqv > L(0.0)) ? rmin(qvap, c.sneqv / DT) : L(0.0);
  T qseva = qvap - qsnsub;
  T qsnfro = (c.sneqv > L(0.0)) ? qdew : L(0.0);
  T qsdew = qdew - qsnfro;

  NMP_PHASE(10);
  // snowwater: func.f90:5049-5174.  Two passes share one copy of `combine`:
  // pass 0 = snowfall + compact + combine, pass 1 = divide + snowh2o head +
  // its conditional combine.
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    bool do_combine;
    if (pass == 0) {
      // snowfall: func.f90:5177-5233
      bool newnode = false;
      if (c.isnow == 0 && c.qsnow > L(0.0)) {
        c.snowh = c.snowh + snowhin * DT;
        c.sneqv = c.sneqv + c.qsnow * DT;
      }
      if (c.isnow == 0 && c.qsnow > L(0.0) && c.snowh >= L(0.025)) {
        c.isnow = -1;
        newnode = true;
        c.dz[2] = c.snowh;
        c.snowh = L(0.0);
        c.stc[2] = rmin(L(273.16), c.sfctmp);
        c.snice[2] = c.sneqv;
        c.snliq[2] = L(0.0);
      }
      if (c.isnow < 0 && !newnode && c.qsnow > L(0.0)) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (j == c.isnow + 3) {
            c.snice[j] = c.snice[j] + c.qsnow * DT;
            c.dz[j] = c.dz[j] + snowhin * DT;
          }
        }
      }
      // compact: func.f90:5580-5677
      if (c.isnow < 0) {
        const T C2 = L(21.e-3), C3 = L(2.5e-6), C4 = L(0.04), C5 = L(2.0), DM = L(100.0);
        const T ETA0 = L(0.8e+6);
        T burden = L(0.0);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (j >= c.isnow + 3) {
            T wx = c.snice[j] + c.snliq[j];
            T fice = c.snice[j] / wx;
            T voidf = L(1.) - (c.snice[j] / DENICE + c.snliq[j] / DENWAT) / c.dz[j];
            if (voidf > L(0.001) && c.snice[j] > L(0.1)) {
              T bi = c.snice[j] / c.dz[j];
              T td = rmax(L(0.0), TFRZ - c.stc[j]);
              T dexpf = M::exp(-C4 * td);
              T ddz1 = -C3 * dexpf;
              if (bi > DM) ddz1 = ddz1 * M::exp(L(-46.0E-3) * (bi - DM));
              if (c.snliq[j] > L(0.01) * c.dz[j]) ddz1 = ddz1 * C5;
              T ddz2 = -(burden + L(0.5) * wx) * M::exp(L(-0.08) * td - C2 * bi) / ETA0;
              T ddz3;
              if (c.imelt[j] == 1) {
                ddz3 = rmax(L(0.0), (c.ficeold[j] - fice) / rmax(L(1.E-6), c.ficeold[j]));
                ddz3 = -ddz3 / DT;
              } else {
                ddz3 = L(0.0);
              }
              T pdzdtc = (ddz1 + ddz2 + ddz3) * DT;
              pdzdtc = rmax(L(-0.5), pdzdtc);
              c.dz[j] = c.dz[j] * (L(1.0) + pdzdtc);
            }
            burden = burden + wx;
          }
        }
      }
      do_combine = c.isnow < 0;
    } else {
      if (c.isnow < 0) divide(c);
      // snowh2o head: func.f90:5726-5766
      if (c.sneqv == L(0.0)) {
        c.sice[0] = c.sice[0] + (qsnfro - qsnsub) * DT / (c.dz[3] * L(1000.0));
        if (c.sice[0] < L(0.0)) {
          c.sh2o[0] = c.sh2o[0] + c.sice[0];
          c.sice[0] = L(0.0);
        }
      }
      if (c.isnow == 0 && c.sneqv > L(0.0)) {
        T temp = c.sneqv;
        c.sneqv = c.sneqv - qsnsub * DT + qsnfro * DT;
        T propor = c.sneqv / temp;
        c.snowh = rmax(L(0.0), propor * c.snowh);
        if (c.sneqv < L(0.0)) {
          c.sice[0] = c.sice[0] + c.sneqv / (c.dz[3] * L(1000.0));
          c.sneqv = L(0.0);
          c.snowh = L(0.0);
        }
        if (c.sice[0] < L(0.0)) {
          c.sh2o[0] = c.sh2o[0] + c.sice[0];
          c.sice[0] = L(0.0);
        }
      }
      if (c.snowh <= L(1.0E-8) || c.sneqv <= L(1.0E-6)) {
        c.snowh = L(0.0);
        c.sneqv = L(0.0);
      }
      do_combine = false;
      if (c.isnow < 0) {
        T wgdif = L(0.0);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (j == c.isnow + 3) {
            wgdif = c.snice[j] - qsnsub * DT + qsnfro * DT;
            c.snice[j] = wgdif;
          }
        }
        do_combine = (wgdif < L(1.0E-6) && c.isnow < 0);
      }
    }
    if (do_combine) combine(c, ponding1, ponding2);
  }
  // snowh2o tail: func.f90:5773-5818
  {
    if (c.isnow < 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (j == c.isnow + 3) {
          c.snliq[j] = c.snliq[j] + qrain * DT;
          c.snliq[j] = rmax(L(0.0), c.snliq[j]);
        }
      }
    }
    T vol_liq[3] = {L(0.), L(0.), L(0.)}, vol_ice[3] = {L(0.), L(0.), L(0.)};
    T epor[3] = {L(0.), L(0.), L(0.)};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j >= c.isnow + 3) {
        vol_ice[j] = rmin(L(1.0), c.snice[j] / (c.dz[j] * DENICE));
        epor[j] = L(1.0) - vol_ice[j];
        vol_liq[j] = rmin(epor[j], c.snliq[j] / (c.dz[j] * DENWAT));
      }
    }
    T qin = L(0.0), qout = L(0.0);
    const T ssi = (T)P.g.ssi;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j >= c.isnow + 3) {
        c.snliq[j] = c.snliq[j] + qin;
        if (j < 2) {
          const int j1 = j < 2 ? j + 1 : 2;
          if (epor[j] < L(0.05) || epor[j1] < L(0.05)) {
            qout = L(0.0);
          } else {
            qout = rmax(L(0.0), (vol_liq[j] - ssi * epor[j]) * c.dz[j]);
            qout = rmin(qout, (L(1.0) - vol_ice[j1] - vol_liq[j1]) * c.dz[j1]);
          }
        } else {
          qout = rmax(L(0.0), (vol_liq[j] - ssi * epor[j]) * c.dz[j]);
        }
        qout = qout * L(1000.0);
        c.snliq[j] = c.snliq[j] - qout;
        qin = qout;
      }
    }
    qsnbot = qout / DT;
  }
  // snowwater tail: empty layers, glacier overflow, layer geometry
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j <= c.isnow + 2) {
      c.snice[j] = L(0.0);
      c.snliq[j] = L(0.0);
      c.stc[j] = L(0.0);
      c.dz[j] = L(0.0);
      c.zsnso[j] = L(0.0);
    }
  }
  if (c.sneqv > L(2000.0)) {
    T bdsnow = c.snice[2] / c.dz[2];
    snoflow = (c.sneqv - L(2000.0));
    c.snice[2] = c.snice[2] - snoflow;
    c.dz[2] = c.dz[2] - snoflow / bdsnow;
    snoflow = snoflow / DT;
  }
  if (c.isnow < 0) {
    c.sneqv = L(0.0);
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j >= c.isnow + 3) c.sneqv = c.sneqv + c.snice[j] + c.snliq[j];
  }
  {
    const int kt2 = c.isnow + 3;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j >= kt2) c.dz[j] = -c.dz[j];
    c.dz[3] = zsoil[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) c.dz[k + 3] = (zsoil[k] - zsoil[k - 1]);
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int km = k > 0 ? k - 1 : 0;
      if (k == kt2)
        c.zsnso[k] = c.dz[k];
      else if (k > kt2)
        c.zsnso[k] = c.zsnso[km] + c.dz[k];
    }
#pragma unroll
    for (int k = 0; k < 7; ++k)
      if (k >= kt2) c.dz[k] = -c.dz[k];
  }
  // snow/soil temperatures, layer geometry and snow layers are final here
  // (soilh2o/groundwater/carbon only read them): store now, free the registers
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    out.s(NMP_S_STC + k, c.stc[k]);
    out.s(NMP_S_ZSNSO + k, c.zsnso[k]);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    out.s(NMP_S_SNICE + k, c.snice[k]);
    out.s(NMP_S_SNLIQ + k, c.snliq[k]);
  }
  out.isn(c.isnow);
  NMP_PHASE(11);
  // frozen ground (:4744-4752)
  if (frozen_ground) {
    c.sice[0] = c.sice[0] + (qsdew - qseva) * DT / (c.dz[3] * L(1000.0));
    qsdew = L(0.0);
    qseva = L(0.0);
    if (c.sice[0] < L(0.0)) {
      c.sh2o[0] = c.sh2o[0] + c.sice[0];
      c.sice[0] = L(0.0);
    }
  }
  T qinsrf = (ponding + ponding1 + ponding2) / DT * L(0.001);
  if (c.isnow == 0)
    qinsrf = qinsrf + (qsnbot + qsdew + qrain) * L(0.001);
  else
    qinsrf = qinsrf + (qsnbot + qsdew) * L(0.001);
  qseva = qseva * L(0.001);
  T etrani[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) etrani[k] = (k < nroot) ? etran * c.btrani[k] * L(0.001) : L(0.0);

  if (c.ist == 2) {
    runsrf = L(0.);
    if (c.wslake >= L(5000.)) runsrf = qinsrf * L(1000.0);
    c.wslake = c.wslake + (qinsrf - qseva) * L(1000.0) * DT - runsrf * DT;
  } else {
    NMP_PHASE(12);
    // soilh2o: func.f90:5822-6048
    T wcnd[4], fcr[4];
    T qdrain = L(0.0), fcrmax = L(0.0);
    T qinfil = L(0.0);
    T rsat = L(0.0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      T ep = rmax(L(1.0E-4), (smcmax - c.sice[k]));
      rsat = rsat + rmax(L(0.0), c.sh2o[k] - ep) * c.dz[k + 3];
      c.sh2o[k] = rmin(ep, c.sh2o[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const T e4 = (sizeof(T) == 4 && R) ? (T)A.c_exp_m4 : M::exp(-L(4.0));
      if (NMP_UNFROZEN_FAST && c.sice[k] == L(0.0)) {
        // no ice: FICE = 0, EXP(-4*(1-FICE)) = EXP(-4) = e4, so FCR = 0 exactly
        fcr[k] = L(0.0);
      } else {
        T fice = rmin(L(1.0), c.sice[k] / smcmax);
        fcr[k] = rmax(L(0.0), M::exp(-L(4.0) * (L(1.0) - fice)) - e4) / (L(1.0) - e4);
      }
    }
    T sicemax = L(0.0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (c.sice[k] > sicemax) sicemax = c.sice[k];
      if (fcr[k] > fcrmax) fcrmax = fcr[k];
    }
    if (o.run == 2) {  // zwteq: func.f90:6051-6100
      T wd1 = L(0.0);
#pragma unroll
      for (int k = 0; k < 4; ++k) wd1 = wd1 + (smcmax - c.sh2o[k]) * c.dz[k + 3];
      T dzfine = L(3.0) * (-zsoil[3]) / (T)100;
      c.zwt = L(-3.0) * zsoil[3] - L(0.001);
      T wd2 = L(0.0);
#pragma unroll 1
      for (int k = 1; k <= 100; ++k) {
        T zfine = (T)k * dzfine;
        T temp = L(1.0) + (c.zwt - zfine) / psisat;
        wd2 = wd2 + smcmax * (L(1.0) - M::pow(temp, L(-1.0) / bexp)) * dzfine;
        if (fabs(wd2 - wd1) <= L(0.01)) {
          c.zwt = zfine;
          break;
        }
      }
      runsub = (L(1.0) - fcrmax) * L(4.0) * ((sizeof(T) == 4 && R) ? (T)P.g.exp_mtimean : M::exp(-(T)P.g.timean)) * M::exp(-L(2.0) * c.zwt);
    }
    if (c.lutyp == P.g.isurban) fcr[0] = L(0.95);
    if (o.run == 1 || o.run == 2) {
      const T fff = (o.run == 1) ? L(6.0) : L(2.0);
      T fsat = (o.run == 1) ? (T)P.g.fsatmax * M::exp(L(-0.5) * fff * (c.zwt - L(2.0)))
                            : (T)P.g.fsatmax * M::exp(L(-0.5) * fff * c.zwt);
      if (qinsrf > L(0.0)) {
        runsrf = qinsrf * ((L(1.0) - fcr[0]) * fsat + fcr[0]);
        qinfil = qinsrf - runsrf;
      }
    }
    if (o.run == 3 && qinsrf > L(0.0)) {  // infil: func.f90:6103-6196
      T dt1 = DT / L(86400.0);
      T smcav = smcmax - smcwlt;
      T dmax1 = -zsoil[0] * smcav;
      T dice = -zsoil[0] * c.sice[0];
      dmax1 = dmax1 * (L(1.0) - (c.sh2o[0] + c.sice[0] - smcwlt) / smcav);
      T dd = dmax1;
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        dice = dice + (zsoil[k - 1] - zsoil[k]) * c.sice[k];
        T dmaxk = (zsoil[k - 1] - zsoil[k]) * smcav;
        dmaxk = dmaxk * (L(1.0) - (c.sh2o[k] + c.sice[k] - smcwlt) / smcav);
        dd = dd + dmaxk;
      }
      T val = (L(1.0) - M::exp(-(T)S.kdt * dt1));
      T ddt = dd * val;
      T px = rmax(L(0.0), qinsrf * DT);
      T infmax = (px * (ddt / (px + ddt))) / DT;
      T fcrl = L(1.0);
      if (dice > L(1.0E-2)) {
        T acrt = L(3.0) * (T)S.frzx / dice;
        T sum = L(1.0);
        sum = sum + (acrt * acrt) / L(2.0);  // J=1: ACRT**2 / 2!
        sum = sum + (acrt) / L(1.0);         // J=2: ACRT**1 / 1
        fcrl = L(1.0) - M::exp(-acrt) * sum;
      }
      infmax = infmax * fcrl;
      T factr = rmax(L(0.01), c.sh2o[0] / smcmax);
      T wcnd1 = (T)S.dksat * M::pow(factr, L(2.0) * bexp + L(3.0));
      infmax = rmax(infmax, wcnd1);
      infmax = rmin(infmax, px);
      runsrf = rmax(L(0.0), qinsrf - infmax);
      qinfil = qinsrf - runsrf;
    }
    if (o.run == 4) {
      T smctot = L(0.0), dztot = L(0.0);
      bool stop = false;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!stop) {
          dztot = dztot + c.dz[k + 3];
          smctot = smctot + c.smc[k] * c.dz[k + 3];
          if (dztot >= L(2.0)) stop = true;
        }
      }
      smctot = smctot / dztot;
      T fsat = M::pow(rmax(L(0.01), smctot / smcmax), L(4.0));
      if (qinsrf > L(0.0)) {
        runsrf = qinsrf * ((L(1.0) - fcr[0]) * fsat + fcr[0]);
        qinfil = qinsrf - runsrf;
      }
    }
    int niter = 1;
    if (o.inf == 1) {
      niter = 3;
      if (qinfil * DT > c.dz[3] * smcmax) niter = niter * 2;
    }
    const T dtfine = DT / (T)niter;
    T qdrain_save = L(0.0);
    const T dwsat = (T)S.dwsat, dksat = (T)S.dksat;
    // The sub-steps divide by the layer thicknesses TEMP1 = ZSOIL(K-1) -
    // ZSOIL(K+1) and DENOM = ZSOIL(K-1) - ZSOIL(K) (srt, func.f90:6238-6276),
    // launch-uniform.  In the fp32 "ref" option-set kernels these divisions
    // use DivFast32 (one reciprocal per thickness for the whole step), which
    // equals IEEE a/b for |b| in [2^-126, 2^126], a = 0 or |a| >= 2^-102, and
    // a normal quotient (tools/fdiv_exhaust.hip).  The thicknesses are checked
    // here once against [2^-20, 2^20]; the numerators (WDF * DDZ of very dry
    // soil is ~1e-32, WFLUX may cancel) are checked per division against
    // a = 0 or [2^-102, 2^100], so the quotient lies in [2^-122, 2^120]
    // (tools/div_proof.py soil_sites).  A lane outside takes IEEE division
    // (an exec-masked branch that no lane usually enters).
#if NMP_SOIL_DIV
    constexpr bool kSoilFast = sizeof(T) == 4 && R && OS != 0;
#else
    constexpr bool kSoilFast = false;
#endif
    typedef std::conditional_t<kSoilFast, DivFast32, DivRef<T>> SoilDiv;
    const SoilDiv sd;
    Recip<T> rtemp[3], rden[4], rnden[4];
    bool soil_ok = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const T den = (k == 0) ? -zsoil[0] : (zsoil[k - 1] - zsoil[k]);
      rden[k] = sd.rec(den);
      rnden[k] = sd.rec(-den);
      soil_ok = soil_ok & (fabs(den) >= L(0x1p-20)) & (fabs(den) <= L(0x1p+20));
      if (k < 3) {
        const T tmp = (k == 0) ? -zsoil[1] : (zsoil[k - 1] - zsoil[k + 1]);
        rtemp[k] = sd.rec(tmp);
        soil_ok = soil_ok & (fabs(tmp) >= L(0x1p-20)) & (fabs(tmp) <= L(0x1p+20));
      }
    }
    auto sdv = [&](T a, const Recip<T>& rb) -> T {
      if constexpr (kSoilFast) {
        T q = sd.div(a, rb);
        const T m = fabs(a);
        const bool in = a == L(0.0) || (m >= L(0x1p-102) && m <= L(0x1p+100));  // NaN: out
        if (__builtin_expect(!soil_ok || !in, 0)) {
          q = a / rb.b;
#ifdef NMP_COUNT_FALLBACK
          atomicAdd(&nmp_fb_reason[25], 1u);  // soil-water division on IEEE
#endif
        }
        return q;
      } else {
        return a / rb.b;
      }
    };
#pragma unroll 1
    for (int it = 1; it <= niter; ++it) {
      // srt: func.f90:6199-6305
      T wdf[4], smx[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // FACTR**(BEXP+2) and FACTR**(2 BEXP+3): one base (pow_pair)
        const T expon1 = bexp + L(2.0), expon2 = L(2.0) * bexp + L(3.0);
        if (o.inf == 1) {  // wdfcnd1
          T factr = rmax(L(0.01), c.smc[k] / smcmax);
          T pw1, pw2;
          pow_pair<T, R>(factr, expon1, expon2, pw1, pw2);
          wdf[k] = dwsat * pw1;
          wdf[k] = wdf[k] * (L(1.0) - fcr[k]);
          wcnd[k] = dksat * pw2;
          wcnd[k] = wcnd[k] * (L(1.0) - fcr[k]);
          smx[k] = c.smc[k];
        } else {  // wdfcnd2
          T factr = rmax(L(0.01), c.sh2o[k] / smcmax);
          T pw1, pw2;
          pow_pair<T, R>(factr, expon1, expon2, pw1, pw2);
          wdf[k] = dwsat * pw1;
          if (sicemax > L(0.0)) {
            T vkwgt = L(1.0) / (L(1.0) + p3(L(500.0) * sicemax));
            wdf[k] = vkwgt * wdf[k] + (L(1.0) - vkwgt) * dwsat * M::pow(L(0.2) / smcmax, expon1);
          }
          wcnd[k] = dksat * pw2;
          smx[k] = c.sh2o[k];
        }
      }
      // DENOM(K) (:6238-6276) is rden[k].b
      T ddz[4], dsmdz[4], wflux[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k == 0) {
          ddz[k] = sdv(L(2.0), rtemp[k]);
          dsmdz[k] = sdv(L(2.0) * (smx[k] - smx[k + 1]), rtemp[k]);
          wflux[k] = wdf[k] * dsmdz[k] + wcnd[k] - qinfil + etrani[k] + qseva;
        } else if (k < 3) {
          ddz[k] = sdv(L(2.0), rtemp[k]);
          dsmdz[k] = sdv(L(2.0) * (smx[k] - smx[k + 1]), rtemp[k]);
          wflux[k] = wdf[k] * dsmdz[k] + wcnd[k] - wdf[k - 1] * dsmdz[k - 1] - wcnd[k - 1] +
                     etrani[k];
        } else {
          if (o.run == 1 || o.run == 2) qdrain = L(0.0);
          if (o.run == 3) qdrain = (T)P.g.slope[c.slptyp - 1] * wcnd[k];
          if (o.run == 4) qdrain = (L(1.0) - fcrmax) * wcnd[k];
          ddz[k] = L(0.0);
          dsmdz[k] = L(0.0);
          wflux[k] = -(wdf[k - 1] * dsmdz[k - 1]) - wcnd[k - 1] + etrani[k] + qdrain;
        }
      }
      T ai[4], bi[4], ci[4], rhstt[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k == 0) {
          ai[k] = L(0.0);
          bi[k] = sdv(wdf[k] * ddz[k], rden[k]);
          ci[k] = -bi[k];
        } else if (k < 3) {
          ai[k] = sdv(-wdf[k - 1] * ddz[k - 1], rden[k]);
          ci[k] = sdv(-wdf[k] * ddz[k], rden[k]);
          bi[k] = -(ai[k] + ci[k]);
        } else {
          ai[k] = sdv(-wdf[k - 1] * ddz[k - 1], rden[k]);
          ci[k] = L(0.0);
          bi[k] = -(ai[k] + ci[k]);
        }
        rhstt[k] = sdv(wflux[k], rnden[k]);
      }
      // sstep: func.f90:6308-6383
      T ciin[4], rin[4], pp[4], del[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        rhstt[k] = rhstt[k] * dtfine;
        ai[k] = ai[k] * dtfine;
        bi[k] = L(1.0) + bi[k] * dtfine;
        ci[k] = ci[k] * dtfine;
        rin[k] = rhstt[k];
        ciin[k] = ci[k];
        pp[k] = L(0.);
        del[k] = L(0.);
      }
      rosr12<T, 4>(pp, ai, bi, ciin, rin, del, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) c.sh2o[k] = c.sh2o[k] + pp[k];
      T wplus = L(0.0);
#pragma unroll
      for (int k = 3; k >= 1; --k) {
        T ep = rmax(L(1.0E-4), smcmax - c.sice[k]);
        wplus = rmax(c.sh2o[k] - ep, L(0.0)) * c.dz[k + 3];
        c.sh2o[k] = rmin(ep, c.sh2o[k]);
        c.sh2o[k - 1] = c.sh2o[k - 1] + wplus / c.dz[k + 2];
      }
      {
        T ep = rmax(L(1.0E-4), smcmax - c.sice[0]);
        wplus = rmax(c.sh2o[0] - ep, L(0.0)) * c.dz[3];
        c.sh2o[0] = rmin(ep, c.sh2o[0]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) c.smc[k] = c.sh2o[k] + c.sice[k];
      rsat = rsat + wplus;
      qdrain_save = qdrain_save + qdrain;
    }
    qdrain = qdrain_save / (T)niter;
    runsrf = runsrf * L(1000.0) + rsat * L(1000.0) / DT;
    qdrain = qdrain * L(1000.0);
    if (o.run == 2) {
      T wtsub = L(0.0);
#pragma unroll
      for (int k = 0; k < 4; ++k) wtsub = wtsub + wcnd[k] * c.dz[k + 3];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        T mh2o = runsub * DT * (wcnd[k] * c.dz[k + 3]) / wtsub;
        c.sh2o[k] = c.sh2o[k] - mh2o / (c.dz[k + 3] * L(1000.0));
      }
    }
    if (o.run != 1) {
      T mliq[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) mliq[k] = c.sh2o[k] * c.dz[k + 3] * L(1000.0);
      const T watmin = L(0.01);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        T xs = (mliq[k] < L(0.0)) ? watmin - mliq[k] : L(0.0);
        mliq[k] = mliq[k] + xs;
        mliq[k + 1] = mliq[k + 1] - xs;
      }
      T xs = (mliq[3] < watmin) ? watmin - mliq[3] : L(0.0);
      mliq[3] = mliq[3] + xs;
      runsub = runsub - xs / DT;
#pragma unroll
      for (int k = 0; k < 4; ++k) c.sh2o[k] = mliq[k] / (c.dz[k + 3] * L(1000.0));
    }
    if (o.run == 1) {
      // groundwater: func.f90:6458-6639
      const T ROUS = L(0.2), CMIC = L(0.20);
      T dzmm[4], znode[4], mliq[4], epg[4], hk[4], smcg[4];
      dzmm[0] = -zsoil[0] * L(1.0E3);
#pragma unroll
      for (int k = 1; k < 4; ++k) dzmm[k] = L(1.0E3) * (zsoil[k - 1] - zsoil[k]);
      znode[0] = -zsoil[0] / L(2.0);
#pragma unroll
      for (int k = 1; k < 4; ++k) znode[k] = -zsoil[k - 1] + L(0.5) * (zsoil[k - 1] - zsoil[k]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        smcg[k] = c.sh2o[k] + c.sice[k];
        mliq[k] = c.sh2o[k] * dzmm[k];
        epg[k] = rmax(L(0.01), smcmax - c.sice[k]);
        hk[k] = L(1.0E3) * wcnd[k];
      }
      int iwt = 3;  // 0-based layer index above the water table
      if (c.zwt <= -zsoil[1])
        iwt = 0;
      else if (c.zwt <= -zsoil[2])
        iwt = 1;
      else if (c.zwt <= -zsoil[3])
        iwt = 2;
      T qdis = (L(1.0) - fcrmax) * L(5.0) * ((sizeof(T) == 4 && R) ? (T)P.g.exp_mtimean : M::exp(-(T)P.g.timean)) * M::exp(-L(6.0) * (c.zwt - L(2.0)));
      // S_NODE is real(8) in the reference (:6501): evaluate the matric potential in fp64
      double s_node = (double)rmin(L(1.0), dget(smcg, iwt) / smcmax);
      s_node = fmax(s_node, (double)0.01f);
      T smpfz = (T)(-((double)(psisat * L(1000.0)) * ::pow(s_node, (double)(-bexp))));
      smpfz = rmax(L(-120000.0), CMIC * smpfz);
      T ka = dget(hk, iwt);
      T znw = dget(znode, iwt);
      T wh_zwt = -c.zwt * L(1.0E3);
      T wh = smpfz - znw * L(1.0E3);
      T qin = -ka * (wh_zwt - wh) / ((c.zwt - znw) * L(1.0E3));
      qin = rmax(L(-10.0) / DT, rmin(L(10.0) / DT, qin));
      c.wt = c.wt + (qin - qdis) * DT;
      if (iwt == 3) {
        c.wa = c.wa + (qin - qdis) * DT;
        c.wt = c.wa;
        c.zwt = (-zsoil[3] + L(25.0)) - c.wa / L(1000.0) / ROUS;
        mliq[3] = mliq[3] - qin * DT;
        mliq[3] = mliq[3] + rmax(L(0.0), c.wa - L(5000.0));
        c.wa = rmin(c.wa, L(5000.0));
      } else {
        if (iwt == 2) {
          c.zwt = -zsoil[3] - (c.wt - ROUS * L(1000.0) * L(25.0)) / (epg[3]) / L(1000.0);
        } else {
          T ws = L(0.0);
#pragma unroll
          for (int k = 1; k < 4; ++k)
            if (k >= iwt + 2) ws = ws + epg[k] * dzmm[k];
          c.zwt = -dget(zsoil, iwt + 1) - (c.wt - ROUS * L(1000.0) * L(25.0) - ws) /
                                              (dget(epg, iwt + 1)) / L(1000.0);
        }
        T wtsub = L(0.0);
#pragma unroll
        for (int k = 0; k < 4; ++k) wtsub = wtsub + hk[k] * dzmm[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) mliq[k] = mliq[k] - qdis * DT * hk[k] * dzmm[k] / wtsub;
      }
      c.zwt = rmax(L(1.5), c.zwt);
      const T watmin = L(0.01);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        T xs = (mliq[k] < L(0.0)) ? watmin - mliq[k] : L(0.0);
        mliq[k] = mliq[k] + xs;
        mliq[k + 1] = mliq[k + 1] - xs;
      }
      T xs = (mliq[3] < watmin) ? watmin - mliq[3] : L(0.0);
      mliq[3] = mliq[3] + xs;
      c.wa = c.wa - xs;
      c.wt = c.wt - xs;
#pragma unroll
      for (int k = 0; k < 4; ++k) c.sh2o[k] = mliq[k] / dzmm[k];
      runsub = qdis;
    }
    if (o.run == 3 || o.run == 4) runsub = runsub + qdrain;
#pragma unroll
    for (int k = 0; k < 4; ++k) c.smc[k] = c.sh2o[k] + c.sice[k];
  }
  runsub = runsub + snoflow;
  // ===================== end water =====================
  // soil water and aquifer are final after the water phase (carbon only reads SMC)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    out.s(NMP_S_SH2O + k, c.sh2o[k]);
    out.s(NMP_S_SMC + k, c.smc[k]);
  }
  out.s(NMP_S_ZWT, c.zwt); out.s(NMP_S_WA, c.wa); out.s(NMP_S_WT, c.wt);
  out.s(NMP_S_WSLAKE, c.wslake);
  out.template d<NMP_D_RUNSRF>(runsrf);
  out.template d<NMP_D_RUNSUB>(runsub);
  out.template d<NMP_D_QSNBOT>(qsnbot);
  out.template d<NMP_D_PONDING1>(ponding1);
  out.template d<NMP_D_PONDING2>(ponding2);

  NMP_PHASE(13);
  // carbon + co2flux (opt_veg 2|5): func.f90:6642-7025
  T gpp = L(0.0), npp = L(0.0), nee = L(0.0);
  if (o.veg == 2 || o.veg == 5) {
    // carbon pools are read and written only when the carbon model runs
    c.lfmass = out.ls(NMP_S_LFMASS); c.rtmass = out.ls(NMP_S_RTMASS);
    c.stmass = out.ls(NMP_S_STMASS); c.wood = out.ls(NMP_S_WOOD);
    c.stblcp = out.ls(NMP_S_STBLCP); c.fastcp = out.ls(NMP_S_FASTCP);
    if (c.lutyp == P.g.iswater || c.lutyp == P.g.isbarren || c.lutyp == P.g.isice ||
        c.lutyp == P.g.isurban) {
      c.lai = c.sai = L(0.0);
      c.lfmass = c.rtmass = c.stmass = c.wood = c.stblcp = c.fastcp = L(0.0);
    } else {
      T lapm = (T)V.sla / L(1000.0);
      T wstres = L(1.0) - btran;
      T wroot = L(0.0);
      const T zr = -(nroot > 0 ? (T)zget(A.zsoil, nroot - 1) : L(1.0));
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < nroot) wroot = wroot + c.smc[k] / smcmax * c.dz[k + 3] / zr;
      const T RTOVRC = L(2.0E-8), RSWOODC = L(3.0E-10), BF = L(0.90), WSTRC = L(100.0);
      const T LAIMIN = L(0.05), XSAMIN = L(0.01);
      T sapm = L(3.0) * L(0.001);
      T lfmsmn = LAIMIN / lapm;
      T stmsmn = XSAMIN / sapm;
      T rf = (igs == L(0.0)) ? L(0.5) : L(1.0);
      T fnf = rmin(c.foln / rmax(L(1.0E-06), (T)V.folnmx), L(1.0));
      T tf = M::pow((T)V.arm, (c.tv - L(298.16)) / L(10.0));
      T resp = (T)V.rmf25 * tf * fnf * c.lai * rf * (L(1.0) - wstres);
      T rsleaf = rmin(c.lfmass / DT, resp * L(12.0E-6));
      T rsroot = (T)V.rmr25 * (c.rtmass * L(1.0E-3)) * tf * rf * L(12.0E-6);
      T rsstem = (T)V.rms25 * (c.stmass * L(1.0E-3)) * tf * rf * L(12.0E-6);
      T rswood = RSWOODC * M::exp(L(0.08) * (c.tv - L(298.16))) * c.wood * (T)V.wdpool;
      T carbfx = psn * L(12.0E-6);
      T leafpt = M::exp(L(0.01) * (L(1.0) - M::exp(L(0.75) * c.lai)) * c.lai);
      if (c.lutyp == P.g.isegblf) leafpt = M::exp(L(0.01) * (L(1.0) - M::exp(L(0.50) * c.lai)) * c.lai);
      T nonlef = L(1.0) - leafpt;
      T stempt = c.lai / L(10.0);
      leafpt = leafpt - stempt;
      T woodf = (c.wood > L(0.0))
                    ? (L(1.0) - M::exp(-BF * ((T)V.wrrat * c.rtmass / c.wood)) / BF) * (T)V.wdpool
                    : L(0.0);
      T rootpt = nonlef * (L(1.0) - woodf);
      T woodpt = nonlef * woodf;
      T lftovr = (T)V.ltovrc * L(1.0E-6) * c.lfmass;
      T sttovr = (T)V.ltovrc * L(1.0E-6) * c.stmass;
      T rttovr = RTOVRC * c.rtmass;
      T wdtovr = L(9.5E-10) * c.wood;
      T sc = M::exp(L(-0.3) * rmax(L(0.0), c.tv - (T)V.tdlef)) * (c.lfmass / L(120.0));
      T sd = M::exp((wstres - L(1.0)) * WSTRC);
      T dielf = c.lfmass * L(1.0E-6) * ((T)V.dilefw * sd + (T)V.dilefc * sc);
      T diest = c.stmass * L(1.0E-6) * ((T)V.dilefw * sd + (T)V.dilefc * sc);
      T fragr = (T)V.fragr;
      T grleaf = rmax(L(0.0), fragr * (leafpt * carbfx - rsleaf));
      T grstem = rmax(L(0.0), fragr * (stempt * carbfx - rsstem));
      T grroot = rmax(L(0.0), fragr * (rootpt * carbfx - rsroot));
      T grwood = rmax(L(0.0), fragr * (woodpt * carbfx - rswood));
      T addnpplf = rmax(L(0.), leafpt * carbfx - grleaf - rsleaf);
      T addnppst = rmax(L(0.), stempt * carbfx - grstem - rsstem);
      if (c.tv < (T)V.tmin) addnpplf = L(0.0);
      if (c.tv < (T)V.tmin) addnppst = L(0.0);
      T lfdel = (c.lfmass - lfmsmn) / DT;
      T stdel = (c.stmass - stmsmn) / DT;
      dielf = rmin(dielf, lfdel + addnpplf - lftovr);
      diest = rmin(diest, stdel + addnppst - sttovr);
      T nppl = rmax(addnpplf, -lfdel);
      T npps = rmax(addnppst, -stdel);
      T nppr = rootpt * carbfx - rsroot - grroot;
      T nppw = woodpt * carbfx - rswood - grwood;
      c.lfmass = c.lfmass + (nppl - lftovr - dielf) * DT;
      c.stmass = c.stmass + (npps - sttovr - diest) * DT;
      c.rtmass = c.rtmass + (nppr - rttovr) * DT;
      if (c.rtmass < L(0.0)) {
        rttovr = nppr;
        c.rtmass = L(0.0);
      }
      c.wood = (c.wood + (nppw - wdtovr) * DT) * (T)V.wdpool;
      c.fastcp = c.fastcp + (rttovr + lftovr + sttovr + wdtovr + dielf) * DT;
      T fst = M::exp2((c.stc[3] - L(283.16)) / L(10.0));
      T fsw = wroot / (L(0.20) + wroot) * L(0.23) / (L(0.23) + wroot);
      T rssoil = fsw * fst * (T)V.mrp * rmax(L(0.0), c.fastcp * L(1.0E-3)) * L(12.0E-6);
      T stablc = L(0.1) * rssoil;
      c.fastcp = c.fastcp - (rssoil + stablc) * DT;
      c.stblcp = c.stblcp + stablc * DT;
      gpp = carbfx;
      npp = nppl + nppw + nppr;
      T autors = rsroot + rswood + rsleaf + grleaf + grroot + grwood;
      T heters = rssoil;
      nee = (autors + heters - gpp) * L(44.0) / L(12.0);
      c.lai = rmax(c.lfmass * lapm, LAIMIN);
      c.sai = rmax(c.stmass * sapm, XSAMIN);
    }
    out.s(NMP_S_LAI, c.lai); out.s(NMP_S_SAI, c.sai);
    out.s(NMP_S_LFMASS, c.lfmass); out.s(NMP_S_RTMASS, c.rtmass);
    out.s(NMP_S_STMASS, c.stmass); out.s(NMP_S_WOOD, c.wood);
    out.s(NMP_S_STBLCP, c.stblcp); out.s(NMP_S_FASTCP, c.fastcp);
  }

  out.template d<NMP_D_NEE>(nee);
  out.template d<NMP_D_GPP>(gpp);
  out.template d<NMP_D_NPP>(npp);
  // urban QSFC (:459-463)
  if (c.lutyp == P.g.isurban) {
    T qfx = etran + ecan + edir;
    c.qsfc = (qfx / rhoair * c.ch) + qair;
    q2b = c.qsfc;
  }
  if (c.snowh <= L(1.0E-6) || c.sneqv <= L(1.0E-3)) {
    c.snowh = L(0.0);
    c.sneqv = L(0.0);
  }
  out.template d<NMP_D_Q2B>(q2b);
  out.s(NMP_S_QSFC, c.qsfc); out.s(NMP_S_SNOWH, c.snowh); out.s(NMP_S_SNEQV, c.sneqv);
  NMP_PHASE(15);
}

// ---------------------------------------------------------------------------
// Occupancy target: 4 waves/SIMD for fp32 (128 VGPRs), 2 for fp64 (256).  With
// the launch tails overlapped by two stream ranges (engine.StreamShards) 4 waves
// measured 1,175 Mcs/s against 1,131 at 3 (168 VGPRs, fewer spills), 921 at 2
// and 930 at 5 (tools/sweep.sh; DESIGN.md "Occupancy").  fp64 on config #5
// (global grid, carbon on): 645 Mcs/s at 2 waves, 534 at 3, 453 at 1 (no
// spills, 378 VGPRs) (tools/configs.sh).
// SMALL: the same kernel at half that occupancy (2 fp32 / 1 fp64, fewer or no
// spills) for launches whose columns cannot fill more wave slots anyway:
// config #2's 65,536 columns are one wave per SIMD (DESIGN.md "Small column
// sets": fp64 0.158 -> 0.150 ms per step, fp32 0.130 -> 0.113).
#ifndef NMP_WAVES_PER_EU
#define NMP_WAVES_PER_EU 4
#endif
#ifndef NMP_WAVES_PER_EU_F64
#define NMP_WAVES_PER_EU_F64 2
#endif
template <class T>
constexpr int waves_per_eu(bool small) {
  return sizeof(T) == 4 ? (small ? NMP_WAVES_PER_EU / 2 : NMP_WAVES_PER_EU)
                        : (small ? (NMP_WAVES_PER_EU_F64 + 1) / 2 : NMP_WAVES_PER_EU_F64);
}
// the LDS layer copy's completion is explicit: LDS-DMA loads count in
// vmcnt, and the "memory" clobber keeps every LDS read of the copied fields
// (NMP_LOAD_COLUMN and the re-read after the flux loops, Sink::fresh_state)
// below the wait
template <class T, bool R>
DEV void lds_copy_wait() {
#if NMP_LDS_EXPLICIT_WAIT
  if constexpr (kPrefetch<T, R>) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}

// The loads of column c0 into `Col<T> c` and the column's output sink `out`,
// declared in the enclosing scope.  The layer state comes from the
// workgroup's LDS copy when kPrefetch (issued by the kernel), the other
// fields from HBM; ALBOLD/TAUSS/QSNOW/SNEQVO are loaded where used (the
// daylight radiation block), QSNOW and SNEQVO reassigned before the water
// phase reads them.  A macro, not a function: the kernel body inlined through
// one more function level compiles to a different schedule, with 61 -> 101
// spilled VGPRs (fp32 run-time math) and 31 -> 79 (fp64).
#define NMP_LOAD_COLUMN(T, R)                                                                \
  Col<T> c;                                                                                  \
  const Sink<T> out{a.diag, a.state, a.ld, a.diag_level, a.static_f, a.static_i, a.forcing,  \
                    a.isnow, a.cost, a.ficeold, c0};                                         \
  c.tv = out.ls(NMP_S_TV); c.tg = out.ls(NMP_S_TG);                                          \
  c.fwet = out.ls(NMP_S_FWET); c.snowh = out.ls(NMP_S_SNOWH);                                \
  c.sneqv = out.ls(NMP_S_SNEQV);                                                             \
  c.lai = out.ls(NMP_S_LAI); c.sai = out.ls(NMP_S_SAI);                                      \
  c.albold = c.tauss = c.qsnow = c.sneqvo = (T)0;                                            \
  c.isnow = gld(out.at(a.isnow, 0));                                                         \
  c.lat = out.lf(NMP_F_LAT); c.zref = out.lf(NMP_F_ZLVL);                                    \
  c.shdfac = out.lf(NMP_F_SHDFAC); c.shdmax = out.lf(NMP_F_SHDMAX);                          \
  c.lutyp = out.li(NMP_I_VEGTYP); c.sltyp = out.li(NMP_I_SOILTYP);                           \
  c.isc = out.li(NMP_I_SOILCOLOR);                                                           \
  c.ist = out.li(NMP_I_IST); c.ice = out.li(NMP_I_ICE);                                      \
  c.sfctmp = out.la(NMP_A_SFCTMP); c.sfcprs = out.la(NMP_A_SFCPRS);                          \
  c.psfc = out.la(NMP_A_PSFC);                                                               \
  c.uu = out.la(NMP_A_UU); c.vv = out.la(NMP_A_VV);                                          \
  c.q2 = out.la(NMP_A_Q2);                                                                   \
  c.soldn = out.la(NMP_A_SOLDN); c.lwdn = out.la(NMP_A_LWDN);                                \
  c.cosz = out.la(NMP_A_COSZ);                                                               \
  c.status = 0;                                                                              \
  {                                                                                          \
    lds_copy_wait<T, R>();                                                                   \
    auto rd = [&](int f) -> T {                                                              \
      if constexpr (kPfEntry<T, R>)                                                          \
        return lds_pool()[f * NMP_BLOCK + threadIdx.x];                                      \
      else                                                                                   \
        return out.ls(f);                                                                    \
    };                                                                                       \
    _Pragma("unroll") for (int k = 0; k < 7; ++k) {                                          \
      c.stc[k] = rd(NMP_S_STC + k);                                                          \
      c.zsnso[k] = rd(NMP_S_ZSNSO + k);                                                      \
    }                                                                                        \
    _Pragma("unroll") for (int k = 0; k < 3; ++k) {                                          \
      c.snice[k] = rd(NMP_S_SNICE + k);                                                      \
      c.snliq[k] = rd(NMP_S_SNLIQ + k);                                                      \
    }                                                                                        \
    _Pragma("unroll") for (int k = 0; k < 4; ++k) {                                          \
      c.sh2o[k] = rd(NMP_S_SH2O + k);                                                        \
      c.smc[k] = rd(NMP_S_SMC + k);                                                          \
    }                                                                                        \
  }

template <class T, bool R, bool SMALL, int OS>
__global__ __launch_bounds__(NMP_BLOCK)
__attribute__((amdgpu_waves_per_eu(waves_per_eu<T>(SMALL))))
void sflx_step_kernel(const DevParams* __restrict__ gparams,
                                                          KArgs<T> a) {
#ifdef NMP_WAVE_TIMING
  const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef NMP_PARAMS_GLOBAL
  const DevParams& sp = *gparams;
#else
  __shared__ __attribute__((aligned(16))) DevParams sp;
  {
    const int4* src = reinterpret_cast<const int4*>(gparams);
    int4* dst = reinterpret_cast<int4*>(&sp);
    constexpr int NW = sizeof(DevParams) / sizeof(int4);
    for (int i = threadIdx.x; i < NW; i += blockDim.x) dst[i] = src[i];
  }
  if constexpr (sizeof(T) == 4 && R) stage_math_tables();
  __syncthreads();
#endif
  int64_t blk = blockIdx.x;
  if (a.order) {
    // re-binned launch: workgroups are dealt round-robin over the 8 XCDs
    // (b and b+8 share one), so map consecutive logical blocks -- one rebin
    // tile's -- onto one XCD: its gathered loads and scattered stores then meet
    // in that XCD's L2 instead of leaving partial lines in eight
    const int64_t per = (int64_t)gridDim.x / 8;
    if (blk < per * 8) blk = (blk % 8) * per + blk / 8;
  }
  // lane -> column: the first cpw lanes of each wave step consecutive columns
  // (cpw = 64: gid = blk * 256 + tid, the plain coalesced map)
  const int lane = threadIdx.x & 63;
  if (lane >= a.cpw) return;
  const int64_t gid = (blk * (NMP_BLOCK / 64) + (threadIdx.x >> 6)) * a.cpw + lane;
  if (gid >= a.ncol) return;
  // re-binned launch: this lane steps column order[gid] (a permutation of the
  // columns; every column is independent, so results do not depend on it)
  const int64_t c0 = a.order ? (int64_t)a.order[gid] : gid;
  const T* st0 = a.state + c0;
  // layer state: through the LDS copy (kPrefetch) or straight from HBM.  The
  // copy is issued first; the column's other fields load while it is in flight
  if constexpr (kPrefetch<T, R>) copy_layers_to_lds(st0, a.ld);
  NMP_LOAD_COLUMN(T, R);
  sflx_column<T, R, OS>(sp, a, c, out);
  if (c.status != 0) *out.at(a.status, 0) |= c.status;
#ifdef NMP_WAVE_TIMING
  {
    const unsigned long long wt1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
      const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID
      const unsigned i = atomicAdd(&nmp_wave_ctr, 1u);
      if (i < NMP_WAVE_REC_MAX) {
        unsigned long long* r = nmp_wave_rec + 4 * (size_t)i;
        r[0] = wt0;
        r[1] = wt1;
        r[2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
        r[3] = (unsigned long long)blockIdx.x |
               ((unsigned long long)(((uintptr_t)a.state >> 8) & 0xffffffffu) << 32);
      }
    }
  }
#endif
}

// launch wrapper of one occupancy instantiation: the kernel of option set os
template <class T, bool R, bool SMALL>
void launch_os(int os, dim3 grid, dim3 block, hipStream_t stream, const DevParams* dparams,
               const KArgs<T>& a) {
  if (os == 1)
    hipLaunchKernelGGL((sflx_step_kernel<T, R, SMALL, 1>), grid, block, 0, stream, dparams, a);
  else if (os == 2)
    hipLaunchKernelGGL((sflx_step_kernel<T, R, SMALL, 2>), grid, block, 0, stream, dparams, a);
  else
    hipLaunchKernelGGL((sflx_step_kernel<T, R, SMALL, 0>), grid, block, 0, stream, dparams, a);
}

// The fp64 half-occupancy (small) kernels live in their own translation unit
// (NMP_TU 9, sflx_kernel_f64s.hip) with MachineLICM on: config #2's
// one-wave-per-SIMD kernel runs +2 % with it, the full-occupancy fp64 kernels
// -9 % (profiles/r05/retune_ab.txt)
#if defined(NMP_TU) && NMP_TU == 8
extern template void launch_os<double, false, true>(int, dim3, dim3, hipStream_t,
                                                    const DevParams*, const KArgs<double>&);
#endif

// launch wrapper (one instantiation per precision / math policy).  os: the
// compiled option set matching the engine's options (0 = read at run time)
template <class T, bool R>
hipError_t launch_sflx(const DevParams* dparams, const KArgs<T>& a, hipStream_t stream,
                       bool small, int os) {
  const int64_t cols_per_block = (int64_t)(NMP_BLOCK / 64) * a.cpw;
  const int64_t grid = (a.ncol + cols_per_block - 1) / cols_per_block;
  const int block = NMP_BLOCK;
  if (grid == 0) return hipSuccess;
  // the fast-math fp32 path has neither a small nor option-set instantiation (code size)
  if constexpr (sizeof(T) == 8 || R) {
    if (small)
      launch_os<T, R, true>(os, dim3((unsigned)grid), dim3(block), stream, dparams, a);
    else
      launch_os<T, R, false>(os, dim3((unsigned)grid), dim3(block), stream, dparams, a);
  } else {
    hipLaunchKernelGGL((sflx_step_kernel<T, R, false, 0>), dim3((unsigned)grid), dim3(block), 0,
                       stream, dparams, a);
  }
  return hipGetLastError();
}

#ifdef NMP_PHASE_TIMING
// this translation unit's phase counters (added to out16; reset if asked)
#define NMP_PC_CAT2(a, b) a##b
#define NMP_PC_CAT(a, b) NMP_PC_CAT2(a, b)
#ifdef NMP_TU
#define NMP_TU_ID NMP_TU
#else
#define NMP_TU_ID 0
#endif
int NMP_PC_CAT(phase_cycles_tu, NMP_TU_ID)(unsigned long long* out16, int reset) {
  unsigned long long v[16];
  if (hipMemcpyFromSymbol(v, HIP_SYMBOL(nmp_phase_cycles), sizeof(v)) != hipSuccess) return -4;
  for (int i = 0; i < 16; ++i) out16[i] += v[i];
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(nmp_phase_cycles), z, sizeof(z)) != hipSuccess) return -4;
  }
  return 0;
}
#if !defined(NMP_TU)
extern "C" int nmp_debug_phase_cycles(unsigned long long* out16, int reset) {
  for (int i = 0; i < 16; ++i) out16[i] = 0;
  return phase_cycles_tu0(out16, reset);
}
#elif NMP_TU == 4
int phase_cycles_tu8(unsigned long long* out16, int reset);
int phase_cycles_tu9(unsigned long long* out16, int reset);
extern "C" int nmp_debug_phase_cycles(unsigned long long* out16, int reset) {
  for (int i = 0; i < 16; ++i) out16[i] = 0;
  int r = phase_cycles_tu4(out16, reset);
  if (!r) r = phase_cycles_tu8(out16, reset);
  return r ? r : phase_cycles_tu9(out16, reset);
}
#endif
#endif



#if defined(NMP_COUNT_FALLBACK) && (!defined(NMP_TU) || NMP_TU == 4)
// (probe builds) lanes that left the range proof's domain and re-ran the
// canopy loop with IEEE division since the last reset
extern "C" long long nmp_debug_fallback_count(int reset, unsigned int* why32) {
  unsigned int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(nmp_fallback_ctr), sizeof(n)) != hipSuccess) return -4;
  if (why32 && hipMemcpyFromSymbol(why32, HIP_SYMBOL(nmp_fb_reason), 32 * sizeof(unsigned int)) !=
                   hipSuccess)
    return -4;
  if (reset) {
    const unsigned int z[32] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(nmp_fallback_ctr), z, sizeof(unsigned int)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(nmp_fb_reason), z, sizeof(z)) != hipSuccess)
      return -4;
  }
  return n;
}
#endif

#if defined(NMP_WAVE_TIMING) && (!defined(NMP_TU) || NMP_TU == 4)
// the fp32 kernels' wave records: copies min(count, max_rec) records of 4 u64
// into out and returns the number recorded since the last reset (may exceed
// the buffer's NMP_WAVE_REC_MAX); reset clears the counter afterwards
extern "C" long long nmp_debug_wave_records(unsigned long long* out, long long max_rec, int reset) {
  unsigned int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(nmp_wave_ctr), sizeof(n)) != hipSuccess) return -4;
  long long k = n < NMP_WAVE_REC_MAX ? n : NMP_WAVE_REC_MAX;
  if (k > max_rec) k = max_rec;
  if (out && k > 0 &&
      hipMemcpyFromSymbol(out, HIP_SYMBOL(nmp_wave_rec), (size_t)k * 4 * sizeof(unsigned long long)) !=
          hipSuccess)
    return -4;
  if (reset) {
    const unsigned int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(nmp_wave_ctr), &z, sizeof(z)) != hipSuccess) return -4;
  }
  return n;
}
#endif

// Instantiations.  The library compiles this file three times (build.py):
// NMP_TU 4 for the fp32 kernels, NMP_TU 8 (sflx_kernel_f64.hip) for the fp64
// ones and NMP_TU 9 (sflx_kernel_f64s.hip) for the fp64 small kernels, each
// with its own flags; without NMP_TU one object holds them all.
#if !defined(NMP_TU) || NMP_TU == 4
template hipError_t launch_sflx<float, true>(const DevParams*, const KArgs<float>&, hipStream_t,
                                             bool, int);
template hipError_t launch_sflx<float, false>(const DevParams*, const KArgs<float>&, hipStream_t,
                                              bool, int);
#endif
#if !defined(NMP_TU) || NMP_TU == 8
template hipError_t launch_sflx<double, false>(const DevParams*, const KArgs<double>&, hipStream_t,
                                               bool, int);
#endif
#if defined(NMP_TU) && NMP_TU == 9
template void launch_os<double, false, true>(int, dim3, dim3, hipStream_t, const DevParams*,
                                             const KArgs<double>&);
#endif

}  // namespace nmp
