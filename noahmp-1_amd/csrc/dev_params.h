// Device-side lookup tables for the sflx kernel.
//
// A compact re-packing of `nmp_params` (the reference module arrays,
// core/module_noahmp_{gen,soil,veg}_param.f90) holding only what the column
// physics reads, grouped per type so that one column's lookups for its
// vegetation / soil type fall in one contiguous record.  The whole struct is
// ~9 KB and is staged into LDS once per workgroup; every lane then gathers its
// own type's fields from LDS with ds_read (per-lane addresses, no HBM traffic).
#pragma once
#include "vege_domain.h"
#include <stdint.h>

#include <cmath>

#include "glibc_math.h"
#include "noahmp_engine.h"

namespace nmp {

struct VegRec {  // one USGS/MODIS vegetation type (veg_param.f90:19-74)
  float xl, rhol[2], rhos[2], taul[2], taus[2];
  float canwmxp, dleaf, z0mvt, hvt, hvb, rcrown, cwpvt;
  float lai12m[12], sai12m[12];
  float sla, dilefc, dilefw, fragr, ltovrc, wrrat, wdpool, tdlef;
  float rgl, hs, rsmax, rsmin, topt;
  float kc25, akc, ko25, ako, vcmx25, avcmx, bp, mp, qe25, folnmx, tmin;
  float rmf25, rms25, rmr25, arm, mrp;
  int32_t nroot, c3c4;
  // 1: the parameters lie in the stomata bisection's proven box
  // (vege_domain.h, tools/div_proof.py), so its divisions may be short
  int32_t stomata_fast, pad_;
  // veg-type-only transcendentals, evaluated once on the host (glibc-exact):
  // twostream AVMU (:2338-2341), LOG(HVT/Z0MVT) (vege_flux UC :2725) and
  // LOG((2+Z0M)/Z0M) (sfcdif1 TMPCM2 :3419 with Z0M = Z0MVT)
  float avmu, log_hvt_z0m, log_2z0m;
};

struct SoilRec {  // one soil type (soil_param.f90:13-23)
  float bexp, smcmax, smcref, smcwlt, psisat, dksat, dwsat, quartz, kdt, frzx;
  // soil-type-only factors of tdfcnd (func.f90:1552-1593), evaluated once on
  // the host with the glibc-exact libm: THKS**(1-SMCMAX) and THKDRY
  float tdf_thks_pow, tdf_thkdry;
  float rsurf_den;  // 2.2E-5*SMCMAX**2*(1-SMCWLT/SMCMAX)**(2+3/BEXP) (rsurf :1150-1151)
  // THKSAT of an unfrozen layer (SH2O == SMC: XU = SMCMAX, TKICE**0 = 1):
  // THKS**(1-SMCMAX) * 1 * THKW**SMCMAX, in tdfcnd's own order (func.f90:1564-1569)
  float tdf_thksat_wet;
  // the same two tdfcnd factors in double for the fp64 path (host libm)
  double tdf_thks_pow_d, tdf_thkdry_d;
};

struct GenRec {  // GENPARMMP.TBL scalars + soil colours (gen_param.f90:12-48, soil_param.f90:27-28)
  float slope[NMP_MSLOPETYP];
  float csoil, zbot, czil, timean, fsatmax, mltfct, z0sno, ssi, swemax;
  float exp_mtimean;  // EXP(-TIMEAN) (groundwater :6531, zwteq), glibc-exact
  float alblake[2], omegas[2], betads, betais, emssoil, emslake;
  float albsat[NMP_MSLCOL][2], albdry[NMP_MSLCOL][2];
  int32_t isurban, iswater, isbarren, isice, isegblf, pad_;
};

// alignas(16): the kernel stages the struct into LDS with int4 copies of
// sizeof/16 chunks, so the size must be a whole number of 16-byte chunks
// (9400 B before this alignment left the last 8 bytes -- veg[26].nroot/c3c4 --
// unstaged).
struct alignas(16) DevParams {
  GenRec g;
  SoilRec soil[NMP_MSLTYP];
  VegRec veg[NMP_MLUTYP];
};

// host copy of the glibc libm tables (glibc_math.h), for host-side precompute
inline const gm::GmTables kHostGmTables = {GM_EXP2F_TAB, GM_LOGF_TAB, GM_POWF_TAB};

inline void pack_dev_params(const nmp_params& p, DevParams& d) {
  for (int i = 0; i < NMP_MSLOPETYP; ++i) d.g.slope[i] = p.slope[i];
  d.g.csoil = p.csoil; d.g.zbot = p.zbot; d.g.czil = p.czil; d.g.timean = p.timean;
  d.g.fsatmax = p.fsatmax; d.g.mltfct = p.mltfct; d.g.z0sno = p.z0sno; d.g.ssi = p.ssi;
  d.g.swemax = p.swemax;
  for (int b = 0; b < 2; ++b) {
    d.g.alblake[b] = p.alblake[b];
    d.g.omegas[b] = p.omegas[b];
  }
  d.g.betads = p.betads; d.g.betais = p.betais; d.g.emssoil = p.emssoil; d.g.emslake = p.emslake;
  for (int c = 0; c < NMP_MSLCOL; ++c)
    for (int b = 0; b < 2; ++b) {
      d.g.albsat[c][b] = p.albsat[c][b];
      d.g.albdry[c][b] = p.albdry[c][b];
    }
  d.g.isurban = p.isurban; d.g.iswater = p.iswater; d.g.isbarren = p.isbarren;
  d.g.isice = p.isice; d.g.isegblf = p.isegblf; d.g.pad_ = 0;
  for (int s = 0; s < NMP_MSLTYP; ++s) {
    SoilRec& r = d.soil[s];
    r.bexp = p.bexp[s]; r.smcmax = p.smcmax[s]; r.smcref = p.smcref[s]; r.smcwlt = p.smcwlt[s];
    r.psisat = p.psisat[s]; r.dksat = p.dksat[s]; r.dwsat = p.dwsat[s]; r.quartz = p.quartz[s];
    r.kdt = p.kdt[s]; r.frzx = p.frzx[s];
    // tdfcnd: THKS = THKQTZ**QZ * 2.0**(1-QZ); THKSAT's first factor THKS**(1-SMCMAX);
    // GAMMD = (1-SMCMAX)*2700; THKDRY = (0.135*GAMMD + 64.7) / (2700 - 0.947*GAMMD)
    const gm::GmTables& T = kHostGmTables;
    const float thks = gm::powf(7.7f, r.quartz, T) * gm::exp2f(1.0f - r.quartz, T);
    r.tdf_thks_pow = gm::powf(thks, 1.0f - r.smcmax, T);
    r.tdf_thksat_wet = (r.tdf_thks_pow * gm::powf(2.2f, 0.0f, T)) * gm::powf(0.57f, r.smcmax, T);
    const float gammd = (1.0f - r.smcmax) * 2700.0f;
    r.tdf_thkdry = (0.135f * gammd + 64.7f) / (2700.0f - 0.947f * gammd);
    {
      const double qz = r.quartz, smx = r.smcmax;
      const double thks_d = std::pow(7.7, qz) * std::exp2(1.0 - qz);
      r.tdf_thks_pow_d = std::pow(thks_d, 1.0 - smx);
      const double gammd_d = (1.0 - smx) * 2700.0;
      r.tdf_thkdry_d = (0.135 * gammd_d + 64.7) / (2700.0 - 0.947 * gammd_d);
    }
    r.rsurf_den = 2.2E-5f * r.smcmax * r.smcmax *
                  gm::powf(1.0f - r.smcwlt / r.smcmax, 2.0f + 3.0f / r.bexp, T);
  }
  d.g.exp_mtimean = gm::expf(-p.timean, kHostGmTables);
  for (int v = 0; v < NMP_MLUTYP; ++v) {
    VegRec& r = d.veg[v];
    r.xl = p.xl[v];
    for (int b = 0; b < 2; ++b) {
      r.rhol[b] = p.rhol[v][b]; r.rhos[b] = p.rhos[v][b];
      r.taul[b] = p.taul[v][b]; r.taus[b] = p.taus[v][b];
    }
    r.canwmxp = p.canwmxp[v]; r.dleaf = p.dleaf[v]; r.z0mvt = p.z0mvt[v]; r.hvt = p.hvt[v];
    r.hvb = p.hvb[v]; r.rcrown = p.rcrown[v]; r.cwpvt = p.cwpvt[v];
    for (int m = 0; m < 12; ++m) {
      r.lai12m[m] = p.lai12m[v][m];
      r.sai12m[m] = p.sai12m[v][m];
    }
    r.sla = p.sla[v]; r.dilefc = p.dilefc[v]; r.dilefw = p.dilefw[v]; r.fragr = p.fragr[v];
    r.ltovrc = p.ltovrc[v]; r.wrrat = p.wrrat[v]; r.wdpool = p.wdpool[v]; r.tdlef = p.tdlef[v];
    r.rgl = p.rgl[v]; r.hs = p.hs[v]; r.rsmax = p.rsmax[v]; r.rsmin = p.rsmin[v]; r.topt = p.topt[v];
    r.kc25 = p.kc25[v]; r.akc = p.akc[v]; r.ko25 = p.ko25[v]; r.ako = p.ako[v];
    r.vcmx25 = p.vcmx25[v]; r.avcmx = p.avcmx[v]; r.bp = p.bp[v]; r.mp = p.mp[v];
    r.qe25 = p.qe25[v]; r.folnmx = p.folnmx[v]; r.tmin = p.tmin[v];
    r.rmf25 = p.rmf25[v]; r.rms25 = p.rms25[v]; r.rmr25 = p.rmr25[v]; r.arm = p.arm[v];
    r.mrp = p.mrp[v];
    r.nroot = p.nroot[v]; r.c3c4 = p.c3c4[v];
    {
      auto in = [](float x, double lo, double hi) { return x >= (float)lo && x <= (float)hi; };
      r.stomata_fast =
          in(r.kc25, NMP_DOM_KC25_LO, NMP_DOM_KC25_HI) && in(r.akc, NMP_DOM_AKC_LO, NMP_DOM_AKC_HI) &&
          in(r.ko25, NMP_DOM_KO25_LO, NMP_DOM_KO25_HI) && in(r.ako, NMP_DOM_AKO_LO, NMP_DOM_AKO_HI) &&
          in(r.avcmx, NMP_DOM_AVCMX_LO, NMP_DOM_AVCMX_HI) && in(r.mp, NMP_DOM_MP_LO, NMP_DOM_MP_HI) &&
          in(r.bp, NMP_DOM_BP_LO, NMP_DOM_BP_HI) &&
          (r.qe25 == 0.0f || in(r.qe25, NMP_DOM_QE25_LO, NMP_DOM_QE25_HI)) &&
          (r.vcmx25 == 0.0f || (in(r.vcmx25, NMP_DOM_VCMX25_LO, NMP_DOM_VCMX25_HI) &&
                                in(r.tmin, NMP_DOM_TMIN_LO, NMP_DOM_TMIN_HI)));
      r.pad_ = 0;
    }
    {
      const gm::GmTables& T = kHostGmTables;
      float chil = r.xl > -0.4f ? r.xl : -0.4f;  // rmin(rmax(XL,-0.4),0.6) as the kernel
      chil = chil < 0.6f ? chil : 0.6f;
      if (__builtin_fabsf(chil) <= 0.01f) chil = 0.01f;
      const float phi1 = 0.5f - 0.633f * chil - 0.330f * chil * chil;
      const float phi2 = 0.877f * (1.0f - 2.0f * phi1);
      r.avmu = (1.0f - phi1 / phi2 * gm::logf((phi1 + phi2) / phi1, T)) / phi2;
      r.log_hvt_z0m = gm::logf(r.hvt / r.z0mvt, T);
      r.log_2z0m = gm::logf((2.0f + r.z0mvt) / r.z0mvt, T);
    }
  }
}

}  // namespace nmp

static_assert(sizeof(nmp::DevParams) % 16 == 0, "DevParams is staged to LDS with int4 copies");
