/*
 * noahmp_engine.h -- C ABI of the MI355X Noah-MP column engine.
 *
 * Drop-in for the reference engine slot `module noahmp_engine`
 * (/root/reference/core/module_noahmp_engine.f90:5-10: empty `noahmp_init`,
 * `noahmp_run`) and for the per-column physics entry it was meant to drive,
 * `noahmp_sflx` (core/module_noahmp_func.f90:66-91, 131 by-reference args).
 *
 * Entry point                 replaces (reference file:line)
 * --------------------------  ------------------------------------------------
 * nmp_read_tables             noahmp_gen_param_readptable   core/module_noahmp_gen_param.f90:51-89
 *                             noahmp_soil_param_readptable  core/module_noahmp_soil_param.f90:31-72
 *                             noahmp_veg_param_readptable   core/module_noahmp_veg_param.f90:77-161
 *                             (block/tag finder             core/module_noahmp_utils.f90:200-237)
 * nmp_init                    noahmp_init                   core/module_noahmp_engine.f90:5-6
 *                             noahmp_set_options            core/module_noahmp_global.f90:77-112
 * nmp_step                    noahmp_run                    core/module_noahmp_engine.f90:8-10
 *                             = noahmp_sflx over every column core/module_noahmp_func.f90:66-476
 * nmp_run, nmp_run_out        the offline time loop around noahmp_run (run/main.py:12-14
 *                             stops after the namelist): many steps, one launch
 * nmp_sflx_columns,           noahmp_sflx itself, argument for argument, on n host records
 *   nmp_sflx_column                                         core/module_noahmp_func.f90:66-476
 * nmp_forcing_from_ldasin,    the forcing arguments of noahmp_sflx (:72-74) from the LDASIN
 *   nmp_forcing_from_ldasin_geo, variables the namelist's input files carry (run/case.nml:6-7)
 *   nmp_ldasin_ingest,
 *   nmp_ldasout_grid         (and the LDASOUT file's grids from the step's diagnostics)
 * nmp_frh2o, nmp_frh2o_host   frh2o (public routine)        core/module_noahmp_func.f90:4494-4598
 * nmp_calhum, nmp_calhum_host calhum (public by default)     core/module_noahmp_func.f90:3958-3984
 * nmp_state_from_aos          layout bridge from noahmp_state_t records
 *                                                           core/module_noahmp_type.f90:10-42
 * nmp_finalize, nmp_strerror  (error path of utils `assert`/`stop`, core/module_noahmp_utils.f90:21-53)
 * nmp_set_launch_variant, nmp_type_size, nmp_option_set, nmp_set_math,
 *   nmp_set_cols_per_wave     engine tuning / host layout checks (no reference counterpart)
 *
 * Conventions
 *  - Plain pointers and sizes only.  All per-column arrays are structure of
 *    arrays, field-major: field f of column c lives at base[f*ld + c]
 *    (ld >= ncol), so one wavefront of 64 lanes reads 64 consecutive columns
 *    of one field per load.  ld < 2^29 (536,870,912 columns per call;
 *    NMP_E_ARG otherwise): the kernel forms a column's byte offset in 32 bits.
 *  - "real" arrays are float when the engine was created with precision 4 and
 *    double with precision 8.  Table values (nmp_params) are always float, as
 *    in the reference (real(r4) module arrays).
 *  - Pointers passed to nmp_step are DEVICE pointers on the engine's device;
 *    `stream` is a hipStream_t (NULL = default stream).  nmp_step only
 *    enqueues work; it never synchronises and never allocates.
 *  - Return codes: 0 ok, negative = NMP_E_*.  Per-column physics failures
 *    that abort the reference (wrf_error_fatal) are reported as NMP_ST_* bits
 *    in col_status instead; the column continues, as the reference code does
 *    after the external returns.
 *  - Threading: one engine per device; calls on one engine are serialised by
 *    the caller.  Engines on different devices/ranks are independent.  The
 *    synchronous host entries (nmp_sflx_columns, nmp_frh2o_host,
 *    nmp_calhum_host) share one device scratch block and stream per engine
 *    and take an engine lock, so concurrent calls of them are safe (they run
 *    one after another).
 */
#ifndef NOAHMP_ENGINE_H
#define NOAHMP_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMP_ABI_VERSION 8

/* ---- dimensions (core/module_noahmp_global.f90:9-13) -------------------- */
#define NMP_NSOIL 4
#define NMP_NSNOW 3
#define NMP_NLAYER 7 /* -NSNOW+1 .. NSOIL ; C index k <-> Fortran index k-2 */
#define NMP_NBAND 2

/* ---- physics options, order = noahmp_set_options (global.f90:77-80) ----- */
typedef struct nmp_options {
  int32_t opt_veg, opt_crs, opt_btr, opt_run, opt_sfc, opt_frz;
  int32_t opt_inf, opt_rad, opt_alb, opt_snf, opt_tbot, opt_stc;
} nmp_options;

/* ---- lookup tables: the reference module arrays, in memory ------------- *
 * Field order == the reference module declarations; 2-D Fortran arrays
 * (band,type) / (month,type) map to C [type][band] / [type][month].
 * Indices are 1-based in the reference: entry i of the C arrays is type i+1. */
#define NMP_MSLOPETYP 30 /* gen_param.f90:8   */
#define NMP_MSLTYP 30    /* soil_param.f90:7  */
#define NMP_MSLCOL 20    /* soil_param.f90:8  */
#define NMP_MLUTYP 27    /* veg_param.f90:8   */

typedef struct nmp_params {
  /* GENPARMMP.TBL  (gen_param.f90:12-48) */
  float slope[NMP_MSLOPETYP];
  float csoil, zbot, czil, dkref, kdtref, frzk, timean, fsatmax;
  float mltfct, z0sno, ssi, swemax;
  float albice[2], alblake[2], omegas[2];
  float betads, betais, emssoil, emslake;
  /* SOILPARMMP.TBL  (soil_param.f90:13-28) */
  float bexp[NMP_MSLTYP], smcmax[NMP_MSLTYP], smcref[NMP_MSLTYP], smcwlt[NMP_MSLTYP];
  float psisat[NMP_MSLTYP], dksat[NMP_MSLTYP], dwsat[NMP_MSLTYP], quartz[NMP_MSLTYP];
  float kdt[NMP_MSLTYP], frzx[NMP_MSLTYP];
  float albsat[NMP_MSLCOL][2], albdry[NMP_MSLCOL][2];
  /* VEGPARMMP.TBL  (veg_param.f90:19-74) */
  float xl[NMP_MLUTYP];
  float rhol[NMP_MLUTYP][2], rhos[NMP_MLUTYP][2], taul[NMP_MLUTYP][2], taus[NMP_MLUTYP][2];
  float canwmxp[NMP_MLUTYP], dleaf[NMP_MLUTYP], z0mvt[NMP_MLUTYP], hvt[NMP_MLUTYP];
  float hvb[NMP_MLUTYP], den[NMP_MLUTYP], rcrown[NMP_MLUTYP], cwpvt[NMP_MLUTYP];
  float sai12m[NMP_MLUTYP][12], lai12m[NMP_MLUTYP][12];
  float sla[NMP_MLUTYP], dilefc[NMP_MLUTYP], dilefw[NMP_MLUTYP], fragr[NMP_MLUTYP];
  float ltovrc[NMP_MLUTYP], wrrat[NMP_MLUTYP], wdpool[NMP_MLUTYP], tdlef[NMP_MLUTYP];
  float rgl[NMP_MLUTYP], hs[NMP_MLUTYP], rsmax[NMP_MLUTYP], rsmin[NMP_MLUTYP], topt[NMP_MLUTYP];
  float kc25[NMP_MLUTYP], akc[NMP_MLUTYP], ko25[NMP_MLUTYP], ako[NMP_MLUTYP];
  float vcmx25[NMP_MLUTYP], avcmx[NMP_MLUTYP], bp[NMP_MLUTYP], mp[NMP_MLUTYP];
  float qe25[NMP_MLUTYP], aqe[NMP_MLUTYP], folnmx[NMP_MLUTYP], tmin[NMP_MLUTYP];
  float rmf25[NMP_MLUTYP], rms25[NMP_MLUTYP], rmr25[NMP_MLUTYP], arm[NMP_MLUTYP], mrp[NMP_MLUTYP];
  float slarea[NMP_MLUTYP], eps[NMP_MLUTYP][5];
  /* integers */
  int32_t nslptyp, nsltyp, nsoilcol, nlutyp;
  int32_t isurban, iswater, isbarren, isice, isegblf; /* veg_param.f90:13-17 */
  int32_t nroot[NMP_MLUTYP], c3c4[NMP_MLUTYP];
} nmp_params;

/* ---- per-column SoA layouts ---------------------------------------------
 * Prognostic fp state (read + written every step).  The first block keeps
 * the snow/soil arrays; index k of a 7-layer field is Fortran layer k-2. */
enum {
  NMP_S_STC = 0,     /* [7] snow/soil temperature (K)              */
  NMP_S_ZSNSO = 7,   /* [7] layer-bottom depth from snow surface (m, <0) */
  NMP_S_SNICE = 14,  /* [3] snow layer ice (mm)                    */
  NMP_S_SNLIQ = 17,  /* [3] snow layer liquid (mm)                 */
  NMP_S_SH2O = 20,   /* [4] soil liquid water (m3/m3) ("soilwat")  */
  NMP_S_SMC = 24,    /* [4] soil total water (m3/m3)               */
  NMP_S_TV = 28, NMP_S_TG, NMP_S_TAH, NMP_S_EAH, NMP_S_FWET, NMP_S_CANLIQ,
  NMP_S_CANICE, NMP_S_QSFC, NMP_S_SNOWH, NMP_S_SNEQV, NMP_S_SNEQVO, NMP_S_ALBOLD,
  NMP_S_TAUSS, NMP_S_QSNOW, NMP_S_ZWT, NMP_S_WA, NMP_S_WT, NMP_S_WSLAKE,
  NMP_S_LAI, NMP_S_SAI, NMP_S_LFMASS, NMP_S_RTMASS, NMP_S_STMASS, NMP_S_WOOD,
  NMP_S_STBLCP, NMP_S_FASTCP, NMP_S_CM, NMP_S_CH,
  NMP_NSTATE = 56 /* + int32 ISNOW in its own array */
};

/* Static fp / int per column (read every step). */
enum { NMP_F_LAT = 0, NMP_F_ZLVL, NMP_F_SHDFAC, NMP_F_SHDMAX, NMP_F_TBOT, NMP_F_FOLN, NMP_NSTATIC_F };
enum { NMP_I_VEGTYP = 0, NMP_I_SOILTYP, NMP_I_SLOPETYP, NMP_I_SOILCOLOR, NMP_I_IST, NMP_I_ICE,
       NMP_NSTATIC_I };

/* Forcing per step (noahmp_sflx :72-74). */
enum { NMP_A_SFCTMP = 0, NMP_A_SFCPRS, NMP_A_PSFC, NMP_A_UU, NMP_A_VV, NMP_A_Q2, NMP_A_SOLDN,
       NMP_A_LWDN, NMP_A_PRCP, NMP_A_COSZ, NMP_A_CO2AIR, NMP_A_O2AIR, NMP_NFORCING };

/* LDASIN forcing block (nmp_forcing_from_ldasin): the 8 variables of an
 * HRLDAS LDASIN file (noahmp-1_amd/ncio.py) plus the step's cosine of the
 * solar zenith angle, always fp32, field-major like every SoA array. */
enum { NMP_L_T2D = 0, NMP_L_Q2D, NMP_L_U2D, NMP_L_V2D, NMP_L_PSFC, NMP_L_RAINRATE, NMP_L_SWDOWN,
       NMP_L_LWDOWN, NMP_L_COSZ, NMP_NLDASIN };

/* Per-column climate record of the synthetic forcing generator
 * (nmp_forcing_synth): latitude / longitude (radians), mean air temperature
 * (K), diurnal amplitude (K), relative humidity (0-1), surface pressure (Pa),
 * mean wind u / v (m/s), precipitation probability per step. */
enum { NMP_CLIM_LAT = 0, NMP_CLIM_LON, NMP_CLIM_T0, NMP_CLIM_AMP, NMP_CLIM_RH, NMP_CLIM_PRES,
       NMP_CLIM_WIND_U, NMP_CLIM_WIND_V, NMP_CLIM_WET, NMP_NCLIM };

/* Full diagnostics = the 58 intent(out) args of noahmp_sflx in dummy order (:82-91). */
enum {
  NMP_D_FSA = 0, NMP_D_FSR, NMP_D_FIRA, NMP_D_FSH, NMP_D_SSOIL, NMP_D_FCEV,
  NMP_D_FGEV, NMP_D_FCTR, NMP_D_ECAN, NMP_D_ETRAN, NMP_D_EDIR, NMP_D_TRAD,
  NMP_D_TGB, NMP_D_TGV, NMP_D_T2MV, NMP_D_T2MB, NMP_D_Q2V, NMP_D_Q2B,
  NMP_D_RUNSRF, NMP_D_RUNSUB, NMP_D_APAR, NMP_D_PSN, NMP_D_SAV, NMP_D_SAG,
  NMP_D_FSNO, NMP_D_NEE, NMP_D_GPP, NMP_D_NPP, NMP_D_FVEG, NMP_D_ALBEDO,
  NMP_D_QSNBOT, NMP_D_PONDING, NMP_D_PONDING1, NMP_D_PONDING2, NMP_D_RSSUN, NMP_D_RSSHA,
  NMP_D_BGAP, NMP_D_WGAP, NMP_D_CHV, NMP_D_CHB, NMP_D_EMISSI,
  NMP_D_SHG, NMP_D_SHC, NMP_D_SHB, NMP_D_EVG, NMP_D_EVB, NMP_D_GHV,
  NMP_D_GHB, NMP_D_IRG, NMP_D_IRC, NMP_D_IRB, NMP_D_TR, NMP_D_EVC,
  NMP_D_CHLEAF, NMP_D_CHUC, NMP_D_CHV2, NMP_D_CHB2, NMP_D_FPICE,
  NMP_NDIAG_FULL = 58
};

/* Output-step surface fluxes, gathered across ranks at output steps. */
enum {
  NMP_O_FSA = 0, NMP_O_FSR, NMP_O_FIRA, NMP_O_FSH, NMP_O_SSOIL, NMP_O_FCEV, NMP_O_FGEV,
  NMP_O_FCTR, NMP_O_ECAN, NMP_O_ETRAN, NMP_O_EDIR, NMP_O_TRAD, NMP_O_RUNSRF, NMP_O_RUNSUB,
  NMP_O_T2M, NMP_O_ALBEDO, NMP_NDIAG_OUT = 16
};

/* diag_level for nmp_step */
enum { NMP_DIAG_NONE = 0, NMP_DIAG_OUT = 1, NMP_DIAG_FULL = 2 };

/* Per-column status bits (replace wrf_error_fatal / wrf_message). */
enum {
  NMP_ST_ERRSW = 1,   /* |SWDOWN-(FSA+FSR)| > 0.01     func.f90:688-710 */
  NMP_ST_ERRENG = 2,  /* |energy residual| > 0.01 W/m2 func.f90:712-721 */
  NMP_ST_FIRE = 4,    /* emitted longwave <= 0         func.f90:1284-1292 */
  NMP_ST_HCAN = 8,    /* HCAN <= ZPD                   func.f90:2726-2738 */
  NMP_ST_ZLVL = 16,   /* ZLVL <= ZPD                   func.f90:3412-3415 */
  NMP_ST_FLERCH = 32, /* Flerchinger fallback (info)   func.f90:4588-4590 */
  NMP_ST_OPTVEG = 64, /* unknown opt_veg               func.f90:375-377 */
  NMP_ST_STOP = 128   /* FIRE|ZLVL as the reference oracle reports them (one message) */
};

/* ---- one column, the reference calling sequence ---------------------------
 * All 131 noahmp_sflx dummy arguments (core/module_noahmp_func.f90:66-91), in
 * dummy-argument order.  Every member is 4 bytes and there is no padding, so a
 * Fortran `type, bind(C)` with the same components in the same order maps onto
 * it 1:1.  Arrays follow the reference bounds in C order:
 * stc/zsnso[k] = Fortran (k-2), ficeold/snice/snliq[j] = (j-2),
 * zsoil/soilwat/smc[k] = (k+1). */
typedef struct nmp_sflx_args {
  /* IN: time/space (:67) */
  int32_t iloc, jloc;
  float lat;
  int32_t yearlen;
  float julian, cosz;
  /* IN: model configuration (:68) */
  float dt, dx, dz8w;
  int32_t nsoil;
  float zsoil[NMP_NSOIL];
  int32_t nsnow;
  /* IN: vegetation / soil characteristics (:69-70) and the unused IZ0TLND (:71) */
  float shdfac, shdmax;
  int32_t slptyp, sltyp, lutyp, ice, ist, isc, iz0tlnd;
  /* IN: forcing (:72-74) */
  float sfctmp, sfcprs, psfc, uu, vv, q2, qc, soldn, lwdn, prcp, tbot, co2air, o2air, foln;
  float ficeold[NMP_NSNOW];
  float pblh, zlvl;
  /* IN/OUT (:75-80) */
  float albold, sneqvo;
  float stc[NMP_NLAYER], soilwat[NMP_NSOIL], smc[NMP_NSOIL];
  float tah, eah, fwet, canliq, canice, tv, tg, qsfc, qsnow;
  int32_t isnow;
  float zsnso[NMP_NLAYER], snowh, sneqv, snice[NMP_NSNOW], snliq[NMP_NSNOW];
  float zwt, wa, wt, wslake, lfmass, rtmass, stmass, wood, stblcp, fastcp, lai, sai;
  float cm, ch, tauss;
  /* OUT (:82-91): the 58 intent(out) arguments, indexed by NMP_D_* */
  float out[NMP_NDIAG_FULL];
  /* OUT: NMP_ST_* bits of this call (what wrf_error_fatal / wrf_message reported) */
  int32_t status;
} nmp_sflx_args;

/* ---- errors -------------------------------------------------------------- */
enum {
  NMP_OK = 0,
  NMP_E_ARG = -1,      /* bad argument / null pointer / ld < ncol          */
  NMP_E_TABLE = -2,    /* table file missing, block not found, parse error */
  NMP_E_OPTION = -3,   /* option value outside the reference's range      */
  NMP_E_DEVICE = -4,   /* HIP error (no device, launch failure)           */
  NMP_E_PRECISION = -5, /* precision not 4 or 8                           */
  NMP_E_CALENDAR = -6   /* julian outside [0, yearlen] (split a run at the
                           year boundary; see nmp_step)                     */
};

typedef struct nmp_engine nmp_engine;

/* Parse GENPARMMP.TBL / SOILPARMMP.TBL / VEGPARMMP.TBL from tbl_dir with the
 * reference's block/tag rules ("&NAME" or "&NAME#TAG").  soil_tag is e.g.
 * "STAS" or "STAS-RUC", veg_tag "USGS" or "MODIFIED_IGBP_MODIS_NOAH".  Every
 * field not present in the tables is NaN, as in the reference (nan4 init). */
int nmp_read_tables(const char* tbl_dir, const char* soil_tag, const char* veg_tag,
                    nmp_params* out);

/* Create an engine on HIP device `device` computing in `precision` (4|8)
 * bytes.  Copies the tables to the device once. */
int nmp_init(const nmp_params* params, const nmp_options* opts, int device, int precision,
             nmp_engine** out);

/* One noahmp_sflx time step for ncol columns (all pointers device, SoA with
 * leading dimension ld).  zsoil[4] (<0, m) and dt are domain-wide; julian /
 * yearlen are the step's calendar position (noahmp_sflx :67), 0 <= julian <=
 * yearlen, else NMP_E_CALENDAR (far enough outside it the reference's
 * phenology reads its monthly LAI/SAI tables out of bounds).  FICEOLD is
 * derived on device from SNICE/SNLIQ at step start, as an offline driver does.
 * diag may be NULL when diag_level == NMP_DIAG_NONE; col_status is OR-ed
 * (caller zeroes it when it wants a fresh mask). */
int nmp_step(nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
             float julian, int32_t yearlen, void* state, int32_t* isnow, const void* static_f,
             const int32_t* static_i, const void* forcing, void* diag, int diag_level,
             int32_t* col_status, void* stream);

/* Column re-binning (no reference counterpart: a scheduling aid for the wave's
 * slowest-lane cost).  nmp_step_binned is nmp_step where lane i
 * steps column order[i] (order: a permutation of 0..ncol-1, device int32, or
 * NULL for the identity) and, when cost is non-NULL, each column's loop-cost
 * key (its vege_flux Newton trip count this step, 0 without a canopy; one byte
 * per column, indexed by column) is written.  Every column reads and writes
 * only its own index in every array, so results are bit-identical for any
 * order.  nmp_rebin builds an order from such keys: within each tile of `tile`
 * consecutive columns (a multiple of 64), the columns sorted by key, so that
 * the waves of the next step hold columns of similar cost.
 * PRECONDITION (not checked by the library): order must be a permutation of
 * 0..ncol-1.  A duplicate entry makes two lanes step the same column at once
 * (a data race on its state) and an entry outside [0, ncol) reads and writes
 * outside the arrays; neither is reported.  Orders built by nmp_rebin satisfy
 * it; the Python Engine.step checks a caller-supplied order when
 * NMP_CHECK_ORDER=1. */
int nmp_step_binned(nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
                    float julian, int32_t yearlen, void* state, int32_t* isnow,
                    const void* static_f, const int32_t* static_i, const void* forcing, void* diag,
                    int diag_level, int32_t* col_status, const int32_t* order, uint8_t* cost,
                    void* stream);
int nmp_rebin(nmp_engine* eng, int64_t ncol, const uint8_t* cost, int32_t* order, int32_t tile,
              void* stream);

/* Same step, many times: nsteps steps (one launch each, enqueued on stream)
 * whose forcing slices are forcing + (s % forcing_period)*forcing_stride
 * (elements, real type; forcing_period 0 = nsteps distinct slices), julian
 * advancing by dt/86400 per step (julian0 + (float)s*dt/86400.0f, every one
 * within [0, yearlen], else NMP_E_CALENDAR: split a run at the year
 * boundary, the next year with its own yearlen, as the reference's driver
 * recomputes the day of year every step);
 * bitwise the same as nsteps nmp_step calls.  diag (if non-NULL) receives the last step only. */
/* Synthetic forcing for one step, generated on the device (no reference
 * counterpart: the reference reads LDASIN files, run/case.nml:6-7, and ships
 * none).  Writes the 12 NMP_A_* fields of ncol columns
 * (SoA, leading dimension ld, engine precision) from their NMP_CLIM_* climate
 * records: a diurnal temperature cycle at local solar time, solar geometry,
 * cloud, humidity, wind and precipitation, with every random draw a
 * counter-based hash of (seed, step, first_col + column, draw).  Stateless:
 * any step of any column can be generated on its own, on any rank. */
int nmp_forcing_synth(nmp_engine* eng, int64_t ncol, int64_t ld, const void* climate,
                      double julian, int32_t yearlen, uint64_t seed, int64_t step,
                      int64_t first_col, void* forcing, void* stream);

/* The 12 NMP_A_* forcing fields of one step (SoA, leading dimension ld,
 * engine precision) from an LDASIN block (fp32, NMP_NLDASIN x ld): the
 * fields noahmp_sflx takes (core/module_noahmp_func.f90:72-74) that the
 * files do not carry are formed on the device -- SFCPRS = PSFC, CO2AIR =
 * 395e-6 PSFC, O2AIR = 0.209 PSFC (one double product rounded to fp32, as the
 * offline driver's host reader forms them) -- so a host uploads 36 B per
 * column per step instead of 48 (fp32) or 96 (fp64).  Device pointers,
 * enqueued on `stream`.  Hosts that supply all 12 fields write the forcing
 * array themselves and skip this call. */
int nmp_forcing_from_ldasin(nmp_engine* eng, int64_t ncol, int64_t ld, const float* ldasin,
                            void* forcing, void* stream);

/* As nmp_forcing_from_ldasin, with COSZ formed on the device instead of read
 * from the block (its NMP_L_COSZ row is not read): geo is (3, ld) double per
 * column -- sin(lat), cos(lat), lon (radians) -- and the step's solar terms
 * come from the host (sin_decl, cos_decl of the declination; ha0 = 2 pi x the
 * UTC fraction of the day).  COSZ = sin_lat sin_decl + (cos_lat cos_decl)
 * cos((ha0 + lon) - pi) in double, rounded once to fp32: the offline driver's
 * host expression (noahmp-1_amd/timeman.py cosz) in its operation order, with
 * the device's double cosine.  A host then uploads an LDASIN file's 8
 * variables once per input interval and nothing on the steps in between. */
int nmp_forcing_from_ldasin_geo(nmp_engine* eng, int64_t ncol, int64_t ld, const float* ldasin,
                                const double* geo, double sin_decl, double cos_decl, double ha0,
                                void* forcing, void* stream);

/* Rows NMP_L_T2D..NMP_L_LWDOWN of an LDASIN block (fp32, leading dimension
 * ld, ncol columns) from the file's own bytes: grid_be holds the 8 variables
 * in NMP_L_* order, each npts grid points of big-endian fp32 as a netCDF-3
 * file stores them, and column c of the block takes grid point point[c]
 * (the land-point selection and the host's column order in one index; a
 * column whose point lies outside [0, npts) gets NaN rows).  The NMP_L_COSZ
 * row is not written.  A host then
 * copies each file's bytes and uploads them; byte order and gather happen
 * here.  Device pointers, enqueued on `stream`. */
int nmp_ldasin_ingest(nmp_engine* eng, int64_t ncol, int64_t ld, int64_t npts,
                      const void* grid_be, const int32_t* point, float* ldasin, void* stream);

/* The output side's mirror: nfield diagnostics of ncol columns (engine
 * precision, field-major, leading dimension ld -- e.g. the NMP_O_* fluxes of
 * nmp_step's diag at level 1) onto the LDASOUT file's grids as a netCDF-3
 * file stores them: grid_be = nfield grids of npts points of big-endian
 * engine-precision reals, `fill` (rounded to the engine precision) where no
 * column lands; column c goes to grid point point[c] (a point outside
 * [0, npts) is skipped).  A host then writes the bytes as they are.  Device
 * pointers, enqueued on `stream`. */
int nmp_ldasout_grid(nmp_engine* eng, int64_t ncol, int64_t ld, int64_t npts, int nfield,
                     const void* diag, const int32_t* point, double fill, void* grid_be,
                     void* stream);

int nmp_run(nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
            float julian0, int32_t yearlen, int32_t nsteps, void* state, int32_t* isnow,
            const void* static_f, const int32_t* static_i, const void* forcing,
            int64_t forcing_stride, int32_t forcing_period, void* diag, int diag_level,
            int32_t* col_status, void* stream);

/* nmp_run with periodic output: every step s with (s+1) % out_every == 0
 * writes its diagnostics (diag_level) to slot ((s+1)/out_every - 1) % diag_slots
 * of the ring diag + slot*diag_stride (elements; >= the diag block size
 * x ld when more than one slot is written).  nmp_run is out_every = nsteps,
 * diag_slots = 1. */
int nmp_run_out(nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
                float julian0, int32_t yearlen, int32_t nsteps, void* state, int32_t* isnow,
                const void* static_f, const int32_t* static_i, const void* forcing,
                int64_t forcing_stride, int32_t forcing_period, void* diag, int diag_level,
                int32_t out_every, int32_t diag_slots, int64_t diag_stride, int32_t* col_status,
                void* stream);

/* Host-side converter: n byte-identical `noahmp_state_t` sequence records
 * (168 B each, core/module_noahmp_type.f90:10-42) -> host SoA float state
 * (ld >= n) + isnow, applying the unit/sign mapping of SURVEY.md 8b.
 * Fields the record lacks are left untouched.
 * PARITY-UNPINNED: no reference code reads or writes noahmp_state_t, so the
 * record's conventions are taken from its field comments alone
 * (core/module_noahmp_type.f90:18,33,41): snowwat is read as mm (kg m-2)
 * although the comment says kg m-3, zsnow as layer tops above ground, zwt as
 * height (+up).  Only the byte layout is tested (tests/test_abi_host.py). */
int nmp_state_from_aos(const void* records, int64_t n, int64_t ld, float* state, int32_t* isnow,
                       int32_t* static_i);

/* noahmp_sflx with the reference calling sequence (func.f90:66-91), for n
 * HOST records: the records are packed into the SoA layout, stepped on the
 * engine's GPU by the same kernel as nmp_step (all 58 outputs), and unpacked
 * in place; synchronous.  Replaces a loop of `call noahmp_sflx(...)` over n
 * columns (the per-column entry SURVEY 8b names nmp_sflx_column).
 *  - nsoil must be 4 and nsnow 3; dt, julian, yearlen and zsoil must be the
 *    same in every record of one call (they are launch-wide), else NMP_E_ARG;
 *    julian outside [0, yearlen] is NMP_E_CALENDAR.
 *  - FICEOLD is taken as the record carries it, like noahmp_sflx's
 *    intent(in) argument (the SoA nmp_step path derives it from SNICE/SNLIQ
 *    at step start instead, as the offline and WRF drivers compute it).
 *  - iloc, jloc, dx, dz8w, qc, pblh and iz0tlnd never enter the arithmetic
 *    (SURVEY H9); zlvl is intent(inout) but never modified, as in the reference.
 *  - status receives the column's NMP_ST_* bits (0 = the reference would not
 *    have called wrf_error_fatal / wrf_message). */
int nmp_sflx_columns(nmp_engine* eng, nmp_sflx_args* cols, int64_t n);
int nmp_sflx_column(nmp_engine* eng, nmp_sflx_args* col);

/* The reference's other public physics routines, batched: element i is one
 * `call frh2o(sltyp(i), FREE(i), TKELV(i), SMC(i), soilwat(i))`
 * (core/module_noahmp_func.f90:4494-4598; public at :6-8) or one
 * `call calhum(SFCTMP(i), SFCPRS(i), Q2SAT(i), DQSDT2(i))` (:3958-3984; a
 * module procedure, public by default).  Reals are the engine's precision;
 * frh2o reads LK_BEXP / LK_PSISAT / LK_SMCMAX of the soil type from the
 * engine's tables, as the reference reads its module arrays.  The device code
 * is the one noahmp_sflx inlines, so in the fp32 "ref" math policy the values
 * are the reference's bit for bit.
 *  - nmp_frh2o / nmp_calhum: device pointers, enqueued on `stream`.
 *  - nmp_frh2o_host / nmp_calhum_host: host arrays, synchronous (copy in,
 *    launch, copy out) -- the drop-in for the scalar Fortran calls (n = 1).
 *  - frh2o: col_status (may be NULL) is OR-ed with NMP_ST_FLERCH where the
 *    reference would call wrf_message (Flerchinger fallback, :4586-4590), and
 *    with NMP_ST_STOP for a soil type outside 1..NMP_MSLTYP (FREE = NaN).
 *  - calhum: q2sat or dqsdt2 may be NULL (not computed). */
int nmp_frh2o(nmp_engine* eng, int64_t n, const int32_t* sltyp, const void* tkelv,
              const void* smc, const void* soilwat, void* free_water, int32_t* col_status,
              void* stream);
int nmp_frh2o_host(nmp_engine* eng, int64_t n, const int32_t* sltyp, const void* tkelv,
                   const void* smc, const void* soilwat, void* free_water, int32_t* col_status);
int nmp_calhum(nmp_engine* eng, int64_t n, const void* sfctmp, const void* sfcprs, void* q2sat,
               void* dqsdt2, void* stream);
int nmp_calhum_host(nmp_engine* eng, int64_t n, const void* sfctmp, const void* sfcprs,
                    void* q2sat, void* dqsdt2);

/* Transcendental policy for fp32 engines: 0 = "ref", a bit-exact restatement of
 * the glibc float libm the reference is linked against (csrc/glibc_math.h;
 * default), 1 = ocml fp32 functions (faster, within a few ulp).  fp64 engines
 * always use ocml double.  Default can also be set with NMP_MATH=fast. */
int nmp_set_math(nmp_engine* eng, int mode);

/* Columns stepped per 64-lane wave: 8..64 (multiple of 8); 0 = 64 (default).
 * Fewer columns per wave spread a small column set over more, partly filled
 * waves; measured slower on config #2, kept as a tuning knob.
 * Results do not depend on it. */
int nmp_set_cols_per_wave(nmp_engine* eng, int cpw);

/* Kernel specialisation for the engine's physics options.  The kernel is
 * compiled for fixed option sets (case.nml's, and case.nml with opt_veg 2);
 * nmp_init picks the one equal to the engine's options, any other combination
 * runs the run-time-options kernel (set 0).  request: -1 = query only,
 * 0 = force the run-time-options kernel, 1 = pick the matching compiled set
 * (the default; env NMP_GENERIC_OPTIONS=1 makes nmp_init start at 0).
 * Returns the set in use (>= 0) or a negative NMP_E_* code.  Results do not
 * depend on it (DESIGN.md "Compile-time option sets"). */
int nmp_option_set(nmp_engine* eng, int request);

/* Occupancy instantiation of the step kernel.  The kernel is compiled twice
 * per option set: at full occupancy (4 waves/SIMD fp32, 2 fp64; spills) and
 * at half occupancy (2 fp32, 1 fp64; fewer or no spills).  NMP_LAUNCH_AUTO
 * (the default) picks the half-occupancy kernel for launches whose waves fit
 * in its slots (csrc/engine.hip small_launch), the full one otherwise;
 * NMP_LAUNCH_SMALL / NMP_LAUNCH_FULL force one for every launch, so a small
 * column set can be pushed through the kernel production sizes run (parity
 * tests of both instantiations).  Env NMP_LAUNCH_VARIANT=auto|small|full sets
 * the default at nmp_init.  Returns the variant in use, or NMP_E_ARG;
 * request -1 only queries.  Results do not depend on it.  The fp32 "fast"
 * math kernel has one instantiation (full) and ignores the setting. */
#define NMP_LAUNCH_AUTO 0
#define NMP_LAUNCH_SMALL 1
#define NMP_LAUNCH_FULL 2
int nmp_set_launch_variant(nmp_engine* eng, int variant);

int nmp_engine_info(const nmp_engine* eng, int* device, int* precision, nmp_options* opts);

/* sizeof of the ABI's records, for hosts that lay them out themselves (a
 * Fortran bind(C) type, a ctypes Structure) and check the layout at start-up:
 * which = NMP_TYPE_PARAMS | NMP_TYPE_OPTIONS | NMP_TYPE_SFLX_ARGS; -1 otherwise. */
#define NMP_TYPE_PARAMS 0
#define NMP_TYPE_OPTIONS 1
#define NMP_TYPE_SFLX_ARGS 2
int64_t nmp_type_size(int which);
void nmp_finalize(nmp_engine* eng);
const char* nmp_strerror(int code);
int nmp_abi_version(void);
/* Hash of the sources and flags this library was compiled from
 * (noahmp-1_amd/build.py source_hash()); the Python loader refuses a library
 * whose hash differs from the sources beside it, so a stale .so never runs. */
const char* nmp_build_hash(void);

#ifdef __cplusplus
}
#endif
#endif /* NOAHMP_ENGINE_H */
