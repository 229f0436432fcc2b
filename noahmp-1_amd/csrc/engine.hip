// C ABI of the MI355X Noah-MP column engine (include/noahmp_engine.h).
//
// Replaces the reference engine slot (core/module_noahmp_engine.f90:5-10) and
// the option setter (core/module_noahmp_global.f90:77-112).  The engine owns
// only the device copy of the lookup tables; every per-column array is
// caller-owned device memory (SoA), so state stays resident in HBM across
// steps and the caller decides streams, graphs and sharding.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "dev_params.h"
#include "noahmp_engine.h"

#include "sflx_kargs.h"

struct nmp_engine {
  int device;
  int precision;
  int math;  // 0 = reference-rounded transcendentals (parity), 1 = fast (fp32 only)
  int cpw;   // columns per wave: 8..64, or 0 = chosen per launch from ncol
  int simds; // SIMDs on the device (CUs x 4)
  int os;    // compiled option set matching opts (sflx_kernel.hip kOptionSet), 0 = none
  int variant;  // NMP_LAUNCH_AUTO | SMALL | FULL: occupancy instantiation per launch
  nmp_options opts;
  nmp::DevParams* dparams;
  // the synchronous host entries (nmp_sflx_columns, nmp_*_host): a private
  // non-blocking stream, so they neither wait for nor stall the caller's
  // streams, and device scratch kept across calls (grown on demand), so a
  // scalar call from a Fortran loop pays no allocation
  hipStream_t hstream;
  char* scratch;
  size_t scratch_bytes;
  // the host entries share hstream and scratch: one at a time per engine
  // (two threads calling them on one engine are serialized here)
  std::mutex host_mu;
};

namespace {

// largest column stride: the kernels form a column's byte offset from a
// field's base in 32 bits (2^29 columns of 8-byte fp64 values = 4 GiB)
constexpr int64_t kMaxColumns = int64_t(1) << 29;

bool options_ok(const nmp_options& o) {
  // valid values of each option (core/module_noahmp_global.f90:17-74)
  return o.opt_veg >= 1 && o.opt_veg <= 5 && o.opt_crs >= 1 && o.opt_crs <= 2 &&
         o.opt_btr >= 1 && o.opt_btr <= 3 && o.opt_run >= 1 && o.opt_run <= 4 &&
         o.opt_sfc >= 1 && o.opt_sfc <= 2 && o.opt_frz >= 1 && o.opt_frz <= 2 &&
         o.opt_inf >= 1 && o.opt_inf <= 2 && o.opt_rad >= 1 && o.opt_rad <= 3 &&
         o.opt_alb >= 1 && o.opt_alb <= 2 && o.opt_snf >= 1 && o.opt_snf <= 3 &&
         o.opt_tbot >= 1 && o.opt_tbot <= 2 && o.opt_stc >= 1 && o.opt_stc <= 2;
}

// the kernel's compiled option sets (sflx_kernel.hip kOptionSet): 1 =
// run/case.nml's options, 2 = the same with opt_veg = 2; 0 = none matches
int option_set(const nmp_options& o) {
  const bool rest = o.opt_crs == 1 && o.opt_btr == 1 && o.opt_run == 1 && o.opt_sfc == 1 &&
                    o.opt_frz == 1 && o.opt_inf == 1 && o.opt_rad == 1 && o.opt_alb == 2 &&
                    o.opt_snf == 1 && o.opt_tbot == 1 && o.opt_stc == 1;
  if (!rest) return 0;
  return o.opt_veg == 1 ? 1 : o.opt_veg == 2 ? 2 : 0;
}

int ensure_device(int dev) {
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return NMP_E_DEVICE;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return NMP_E_DEVICE;
  return NMP_OK;
}

// Device scratch of at least nb bytes for a synchronous host entry (the
// previous contents are not kept).  Growing frees the old block after the
// engine's host stream has drained it.
char* host_scratch(nmp_engine* e, size_t nb) {
  if (nb <= e->scratch_bytes) return e->scratch;
  if (e->scratch) {
    (void)hipStreamSynchronize(e->hstream);
    (void)hipFree(e->scratch);
    e->scratch = nullptr;
    e->scratch_bytes = 0;
  }
  const size_t want = nb < (1u << 20) ? (size_t)(1u << 20) : nb + nb / 4;
  void* p = nullptr;
  if (hipMalloc(&p, want) != hipSuccess) return nullptr;
  e->scratch = static_cast<char*>(p);
  e->scratch_bytes = want;
  return e->scratch;
}

// Columns per wave: 64 unless set.  Fewer columns per wave (more, partly
// filled waves for a small column set) was measured slower on config #2
// (65,536 fp64 columns: 0.158 ms per step at 64, 0.209 at 32, 0.361 at 16,
// DESIGN.md "Small column sets"): the step is not purely latency-bound there.
int cols_per_wave(const nmp_engine* e, int64_t /*ncol*/) { return e->cpw ? e->cpw : 64; }

// Small launches take the half-occupancy kernel (sflx_kernel.hip SMALL): a
// launch whose waves fit in the slots that kernel leaves (one fp64 / two fp32
// waves per SIMD) gains nothing from the higher occupancy and pays its spills.
bool small_launch(const nmp_engine* e, int64_t ncol) {
  if (e->variant == NMP_LAUNCH_SMALL) return true;
  if (e->variant == NMP_LAUNCH_FULL) return false;
  const int64_t waves = (ncol + cols_per_wave(e, ncol) - 1) / cols_per_wave(e, ncol);
  return waves <= (int64_t)e->simds * (e->precision == 4 ? 2 : 1);
}

template <class T>
void fill_args(nmp::KArgs<T>& a, const nmp_engine* e, int64_t ncol, int64_t ld,
               const float zsoil[4], float dt, float julian, int32_t yearlen, void* state,
               int32_t* isnow, const void* sf, const int32_t* si, const void* fc, void* diag,
               int diag_level, int32_t* status, const int32_t* order, uint8_t* cost,
               const void* ficeold) {
  a.ncol = ncol;
  a.ld = ld;
  for (int k = 0; k < 4; ++k) a.zsoil[k] = zsoil[k];
  a.dt = dt;
  a.julian = julian;
  a.yearlen = yearlen;
  a.diag_level = diag_level;
  // launch-uniform transcendentals of the fp32 "ref" path, evaluated once on the
  // host with the same glibc-exact code the kernel runs (csrc/glibc_math.h)
  a.c_exp_m4 = gm::expf(-4.0f, nmp::kHostGmTables);                 // soilh2o FCR :5900-5904
  a.c_albdecay = gm::expf(-0.01f * dt / 3600.0f, nmp::kHostGmTables);  // snowalb_class :2130
  const nmp_options& o = e->opts;
  a.o = nmp::Opt{o.opt_veg, o.opt_crs, o.opt_btr, o.opt_run, o.opt_sfc, o.opt_frz,
                 o.opt_inf, o.opt_rad, o.opt_alb, o.opt_snf, o.opt_tbot, o.opt_stc};
  a.state = static_cast<T*>(state);
  a.isnow = isnow;
  a.static_f = static_cast<const T*>(sf);
  a.static_i = si;
  a.forcing = static_cast<const T*>(fc);
  a.diag = static_cast<T*>(diag);
  a.status = status;
  a.order = order;
  a.cost = cost;
  a.ficeold = static_cast<const T*>(ficeold);
  a.cpw = cols_per_wave(e, ncol);
#ifdef NMP_TRUNC_RUNTIME
  // (probe builds) env NMP_TRUNC_AT: the phase mark the step returns at
  static const int trunc_at = std::getenv("NMP_TRUNC_AT") ? std::atoi(std::getenv("NMP_TRUNC_AT")) : 99;
  a.trunc_at = trunc_at;
#endif
}

int launch(nmp_engine* e, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
           float julian, int32_t yearlen, void* state, int32_t* isnow, const void* sf,
           const int32_t* si, const void* fc, void* diag, int diag_level, int32_t* status,
           hipStream_t stream, const int32_t* order = nullptr, uint8_t* cost = nullptr,
           const void* ficeold = nullptr) {
  // the kernel addresses a column as a 32-bit byte offset from each field's
  // base (sflx_kernel.hip col_at): column indices below kMaxColumns
  if (ld >= kMaxColumns) return NMP_E_ARG;
  hipError_t err;
  if (e->precision == 4) {
    nmp::KArgs<float> a;
    fill_args(a, e, ncol, ld, zsoil, dt, julian, yearlen, state, isnow, sf, si, fc, diag,
              diag_level, status, order, cost, ficeold);
    const bool small = small_launch(e, ncol);
    err = (e->math == 0) ? nmp::launch_sflx<float, true>(e->dparams, a, stream, small, e->os)
                         : nmp::launch_sflx<float, false>(e->dparams, a, stream, small, 0);
  } else {
    nmp::KArgs<double> a;
    fill_args(a, e, ncol, ld, zsoil, dt, julian, yearlen, state, isnow, sf, si, fc, diag,
              diag_level, status, order, cost, ficeold);
    err = nmp::launch_sflx<double, false>(e->dparams, a, stream, small_launch(e, ncol), e->os);
  }
  return err == hipSuccess ? NMP_OK : NMP_E_DEVICE;
}

// The calendar position noahmp_sflx accepts: 0 <= julian <= yearlen (NaN
// fails).  The reference's phenology forms T = 12*DAY/YEARLEN and
// IT1 = T + 0.5 (integer assignment, truncation), IT2 = IT1 + 1, then wraps
// only IT1 < 1 -> 12 and IT2 > 12 -> 1 (func.f90:588-594); DAY = JULIAN in the
// northern hemisphere.  From DAY >= 12.5/12 YEARLEN on, IT1 = 13 indexes
// LK_LAI12M(13, ...) out of bounds (and below -1.5/12 YEARLEN IT2 = 0), so a
// step there has no defined result.  The check is the calendar's own range,
// which also keeps a multi-step run from drifting past the year's end
// unnoticed: the caller splits the run at the boundary with the next year's
// yearlen, as the reference's driver recomputes the day of year every step.
bool julian_ok(float julian, int32_t yearlen) {
  return julian >= 0.0f && julian <= (float)yearlen;
}

int check_common(const nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
                 int32_t yearlen, const void* state, const int32_t* isnow, const void* static_f,
                 const int32_t* static_i, const void* forcing, const void* diag, int diag_level,
                 const int32_t* col_status) {
  if (!zsoil || ld < ncol || !state || !isnow || !static_f || !static_i || !forcing || !col_status)
    return NMP_E_ARG;
  if (ld >= kMaxColumns) return NMP_E_ARG;
  if (diag_level < NMP_DIAG_NONE || diag_level > NMP_DIAG_FULL) return NMP_E_ARG;
  if (diag_level != NMP_DIAG_NONE && !diag) return NMP_E_ARG;
  if (!(dt > 0.0f) || yearlen <= 0) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return NMP_OK;
}

}  // namespace

extern "C" {

int nmp_abi_version(void) { return NMP_ABI_VERSION; }

#ifndef NMP_BUILD_HASH
#define NMP_BUILD_HASH "unknown"
#endif
// the marker prefix lets build.py read the hash from the file without loading it
static const char kBuildHash[] = "NMP_BUILD_HASH=" NMP_BUILD_HASH;
const char* nmp_build_hash(void) { return kBuildHash + 15; }

const char* nmp_strerror(int code) {
  switch (code) {
    case NMP_OK: return "ok";
    case NMP_E_ARG: return "invalid argument";
    case NMP_E_TABLE: return "parameter table missing or unreadable";
    case NMP_E_OPTION: return "physics option out of range";
    case NMP_E_DEVICE: return "HIP device error";
    case NMP_E_PRECISION: return "precision must be 4 or 8";
    case NMP_E_CALENDAR:
      return "julian outside [0, yearlen]: split the run at the year boundary";
    default: return "unknown error";
  }
}

int nmp_init(const nmp_params* params, const nmp_options* opts, int device, int precision,
             nmp_engine** out) {
  if (!params || !opts || !out) return NMP_E_ARG;
  *out = nullptr;
  if (precision != 4 && precision != 8) return NMP_E_PRECISION;
  if (!options_ok(*opts)) return NMP_E_OPTION;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return NMP_E_DEVICE;
  if (ensure_device(device) != NMP_OK) return NMP_E_DEVICE;
  nmp::DevParams host{};
  std::memset(&host, 0, sizeof(host));
  nmp::pack_dev_params(*params, host);
  nmp::DevParams* d = nullptr;
  if (hipMalloc(&d, sizeof(nmp::DevParams)) != hipSuccess) return NMP_E_DEVICE;
  if (hipMemcpy(d, &host, sizeof(host), hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(d);
    return NMP_E_DEVICE;
  }
  nmp_engine* e = new (std::nothrow) nmp_engine;
  if (!e) {
    hipFree(d);
    return NMP_E_ARG;
  }
  e->device = device;
  e->precision = precision;
  const char* m = std::getenv("NMP_MATH");
  e->math = (m && std::strcmp(m, "fast") == 0) ? 1 : 0;
  e->cpw = 0;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  e->simds = 4 * ncu;
  e->opts = *opts;
  // NMP_GENERIC_OPTIONS=1: always the run-time-options kernel (A/B tests, timing)
  const char* g = std::getenv("NMP_GENERIC_OPTIONS");
  e->os = (g && std::strcmp(g, "1") == 0) ? 0 : option_set(*opts);
  // NMP_LAUNCH_VARIANT=small|full: force one occupancy instantiation (parity tests)
  const char* lv = std::getenv("NMP_LAUNCH_VARIANT");
  e->variant = !lv                          ? NMP_LAUNCH_AUTO
               : std::strcmp(lv, "small") == 0 ? NMP_LAUNCH_SMALL
               : std::strcmp(lv, "full") == 0  ? NMP_LAUNCH_FULL
                                               : NMP_LAUNCH_AUTO;
  e->dparams = d;
  e->scratch = nullptr;
  e->scratch_bytes = 0;
  if (hipStreamCreateWithFlags(&e->hstream, hipStreamNonBlocking) != hipSuccess) {
    hipFree(d);
    delete e;
    return NMP_E_DEVICE;
  }
  *out = e;
  return NMP_OK;
}

int nmp_set_math(nmp_engine* eng, int mode) {
  if (!eng || mode < 0 || mode > 1) return NMP_E_ARG;
  eng->math = mode;
  return NMP_OK;
}

int nmp_set_cols_per_wave(nmp_engine* eng, int cpw) {
  if (!eng || cpw < 0 || cpw > 64 || cpw % 8 != 0) return NMP_E_ARG;
  eng->cpw = cpw;
  return NMP_OK;
}

int nmp_option_set(nmp_engine* eng, int request) {
  if (!eng || request < -1 || request > 1) return NMP_E_ARG;
  if (request == 0) eng->os = 0;
  if (request == 1) eng->os = option_set(eng->opts);
  return eng->os;
}

int nmp_set_launch_variant(nmp_engine* eng, int variant) {
  if (!eng || variant < -1 || variant > NMP_LAUNCH_FULL) return NMP_E_ARG;
  if (variant >= 0) eng->variant = variant;
  return eng->variant;
}

int64_t nmp_type_size(int which) {
  switch (which) {
    case NMP_TYPE_PARAMS: return (int64_t)sizeof(nmp_params);
    case NMP_TYPE_OPTIONS: return (int64_t)sizeof(nmp_options);
    case NMP_TYPE_SFLX_ARGS: return (int64_t)sizeof(nmp_sflx_args);
    default: return -1;
  }
}

int nmp_engine_info(const nmp_engine* eng, int* device, int* precision, nmp_options* opts) {
  if (!eng) return NMP_E_ARG;
  if (device) *device = eng->device;
  if (precision) *precision = eng->precision;
  if (opts) *opts = eng->opts;
  return NMP_OK;
}

int nmp_step(nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
             float julian, int32_t yearlen, void* state, int32_t* isnow, const void* static_f,
             const int32_t* static_i, const void* forcing, void* diag, int diag_level,
             int32_t* col_status, void* stream) {
  if (!eng || ncol < 0) return NMP_E_ARG;
  if (ncol == 0) return NMP_OK;
  if (!julian_ok(julian, yearlen)) return NMP_E_CALENDAR;
  int rc = check_common(eng, ncol, ld, zsoil, dt, yearlen, state, isnow, static_f, static_i,
                        forcing, diag, diag_level, col_status);
  if (rc != NMP_OK) return rc;
  return launch(eng, ncol, ld, zsoil, dt, julian, yearlen, state, isnow, static_f, static_i,
                forcing, diag, diag_level, col_status, static_cast<hipStream_t>(stream));
}

int nmp_step_binned(nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
                    float julian, int32_t yearlen, void* state, int32_t* isnow,
                    const void* static_f, const int32_t* static_i, const void* forcing, void* diag,
                    int diag_level, int32_t* col_status, const int32_t* order, uint8_t* cost,
                    void* stream) {
  if (!eng || ncol < 0) return NMP_E_ARG;
  if (ncol == 0) return NMP_OK;
  if (ncol > INT32_MAX && order) return NMP_E_ARG;  // order holds int32 column indices
  if (!julian_ok(julian, yearlen)) return NMP_E_CALENDAR;
  int rc = check_common(eng, ncol, ld, zsoil, dt, yearlen, state, isnow, static_f, static_i,
                        forcing, diag, diag_level, col_status);
  if (rc != NMP_OK) return rc;
  return launch(eng, ncol, ld, zsoil, dt, julian, yearlen, state, isnow, static_f, static_i,
                forcing, diag, diag_level, col_status, static_cast<hipStream_t>(stream), order,
                cost);
}

int nmp_rebin(nmp_engine* eng, int64_t ncol, const uint8_t* cost, int32_t* order, int32_t tile,
              void* stream) {
  if (!eng || ncol < 0 || !cost || !order || ncol > INT32_MAX) return NMP_E_ARG;
  if (tile < 64 || tile > (1 << 20) || tile % 64 != 0) return NMP_E_ARG;
  if (ncol == 0) return NMP_OK;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return nmp::launch_rebin(cost, order, ncol, tile, static_cast<hipStream_t>(stream)) ==
                 hipSuccess
             ? NMP_OK
             : NMP_E_DEVICE;
}

int nmp_forcing_synth(nmp_engine* eng, int64_t ncol, int64_t ld, const void* climate,
                      double julian, int32_t yearlen, uint64_t seed, int64_t step,
                      int64_t first_col, void* forcing, void* stream) {
  if (!eng || ncol < 0 || ld < ncol || yearlen <= 0 || step < 0 || first_col < 0) return NMP_E_ARG;
  if (ncol == 0) return NMP_OK;
  if (!climate || !forcing) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return nmp::launch_forcing_synth(eng->precision, ncol, ld, climate, julian, yearlen, seed, step,
                                   first_col, forcing, static_cast<hipStream_t>(stream)) ==
                 hipSuccess
             ? NMP_OK
             : NMP_E_DEVICE;
}

int nmp_forcing_from_ldasin(nmp_engine* eng, int64_t ncol, int64_t ld, const float* ldasin,
                            void* forcing, void* stream) {
  if (!eng || ncol < 0 || ld < ncol || ld >= kMaxColumns) return NMP_E_ARG;
  if (ncol == 0) return NMP_OK;
  if (!ldasin || !forcing) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return nmp::launch_forcing_ldasin(eng->precision, ncol, ld, ldasin, nullptr, 0.0, 0.0, 0.0,
                                    forcing, static_cast<hipStream_t>(stream)) == hipSuccess
             ? NMP_OK
             : NMP_E_DEVICE;
}

int nmp_ldasin_ingest(nmp_engine* eng, int64_t ncol, int64_t ld, int64_t npts,
                      const void* grid_be, const int32_t* point, float* ldasin, void* stream) {
  if (!eng || ncol < 0 || ld < ncol || ld >= kMaxColumns || npts < 0 || npts >= kMaxColumns)
    return NMP_E_ARG;
  if (ncol == 0) return NMP_OK;
  if (!grid_be || !point || !ldasin || npts == 0) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return nmp::launch_ldasin_ingest(ncol, ld, npts, grid_be, point, ldasin,
                                   static_cast<hipStream_t>(stream)) == hipSuccess
             ? NMP_OK
             : NMP_E_DEVICE;
}

int nmp_ldasout_grid(nmp_engine* eng, int64_t ncol, int64_t ld, int64_t npts, int nfield,
                     const void* diag, const int32_t* point, double fill, void* grid_be,
                     void* stream) {
  if (!eng || ncol < 0 || ld < ncol || ld >= kMaxColumns || npts < 0 || npts >= kMaxColumns ||
      nfield < 0 || nfield > NMP_NDIAG_FULL)
    return NMP_E_ARG;
  if (npts == 0 || nfield == 0) return NMP_OK;
  if (!grid_be || (ncol > 0 && (!diag || !point))) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return nmp::launch_ldasout_grid(eng->precision, ncol, ld, npts, nfield, diag, point, fill,
                                  grid_be, static_cast<hipStream_t>(stream)) == hipSuccess
             ? NMP_OK
             : NMP_E_DEVICE;
}

int nmp_forcing_from_ldasin_geo(nmp_engine* eng, int64_t ncol, int64_t ld, const float* ldasin,
                                const double* geo, double sin_decl, double cos_decl, double ha0,
                                void* forcing, void* stream) {
  if (!eng || ncol < 0 || ld < ncol || ld >= kMaxColumns) return NMP_E_ARG;
  if (ncol == 0) return NMP_OK;
  if (!ldasin || !geo || !forcing) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return nmp::launch_forcing_ldasin(eng->precision, ncol, ld, ldasin, geo, sin_decl, cos_decl, ha0,
                                    forcing, static_cast<hipStream_t>(stream)) == hipSuccess
             ? NMP_OK
             : NMP_E_DEVICE;
}

int nmp_run(nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
            float julian0, int32_t yearlen, int32_t nsteps, void* state, int32_t* isnow,
            const void* static_f, const int32_t* static_i, const void* forcing,
            int64_t forcing_stride, int32_t forcing_period, void* diag, int diag_level,
            int32_t* col_status, void* stream) {
  // diagnostics of the last step only = one output every nsteps steps, one slot
  return nmp_run_out(eng, ncol, ld, zsoil, dt, julian0, yearlen, nsteps, state, isnow, static_f,
                     static_i, forcing, forcing_stride, forcing_period, diag, diag_level,
                     nsteps > 0 ? nsteps : 1, 1, 0, col_status, stream);
}

int nmp_run_out(nmp_engine* eng, int64_t ncol, int64_t ld, const float zsoil[4], float dt,
                float julian0, int32_t yearlen, int32_t nsteps, void* state, int32_t* isnow,
                const void* static_f, const int32_t* static_i, const void* forcing,
                int64_t forcing_stride, int32_t forcing_period, void* diag, int diag_level,
                int32_t out_every, int32_t diag_slots, int64_t diag_stride, int32_t* col_status,
                void* stream) {
  if (!eng || ncol < 0 || nsteps < 0 || forcing_stride < 0 || forcing_period < 0)
    return NMP_E_ARG;
  if (out_every < 1 || diag_slots < 1 || diag_stride < 0) return NMP_E_ARG;
  if (ncol == 0 || nsteps == 0) return NMP_OK;
  // forcing slices and diag slots must not overlap the columns they follow
  const int32_t nslices = forcing_period > 0 ? forcing_period : nsteps;
  if (nslices > 1 && forcing_stride < NMP_NFORCING * ld) return NMP_E_ARG;
  const int32_t nout = nsteps / out_every;
  if (diag_level != NMP_DIAG_NONE && nout > 1 && diag_slots > 1) {
    const int64_t nd = diag_level == NMP_DIAG_FULL ? NMP_NDIAG_FULL : NMP_NDIAG_OUT;
    if (diag_stride < nd * ld) return NMP_E_ARG;
  }
  // every step's julian (formed below exactly as the launches form it) in range
  if (!julian_ok(julian0, yearlen) ||
      !julian_ok(julian0 + (float)(nsteps - 1) * dt / 86400.0f, yearlen))
    return NMP_E_CALENDAR;
  int rc = check_common(eng, ncol, ld, zsoil, dt, yearlen, state, isnow, static_f, static_i,
                        forcing, diag, diag_level, col_status);
  if (rc != NMP_OK) return rc;
  // One launch per step, enqueued back to back on `stream`.  (A single
  // multi-step launch that keeps each block on its columns for all steps was
  // measured slower on the mixed-column benchmark: per-block cost differences
  // persist across steps, whereas per-step launches rebalance blocks over CUs
  // every step -- DESIGN.md "Launch structure".)
  const size_t esz = eng->precision == 4 ? 4 : 8;
  const auto hs = static_cast<hipStream_t>(stream);
  for (int32_t s = 0; s < nsteps; ++s) {
    const int32_t fs = forcing_period > 0 ? s % forcing_period : s;
    const char* f = static_cast<const char*>(forcing) + (size_t)fs * forcing_stride * esz;
    const float jul = julian0 + (float)s * dt / 86400.0f;
    const bool out = diag_level != NMP_DIAG_NONE && (s + 1) % out_every == 0;
    char* d = out ? static_cast<char*>(diag) +
                        (size_t)(((s + 1) / out_every - 1) % diag_slots) * diag_stride * esz
                  : nullptr;
    rc = launch(eng, ncol, ld, zsoil, dt, jul, yearlen, state, isnow, static_f, static_i, f, d,
                out ? diag_level : NMP_DIAG_NONE, col_status, hs);
    if (rc != NMP_OK) return rc;
  }
  return NMP_OK;
}

int nmp_state_from_aos(const void* records, int64_t n, int64_t ld, float* state, int32_t* isnow,
                       int32_t* static_i) {
  // noahmp_state_t: 42 x 4-byte sequence record (core/module_noahmp_type.f90:10-42)
  if (!records || n < 0 || ld < n || !state || !isnow) return NMP_E_ARG;
  const unsigned char* base = static_cast<const unsigned char*>(records);
  for (int64_t c = 0; c < n; ++c) {
    float w[42];
    std::memcpy(w, base + c * 168, 168);
    int32_t lutyp, sltyp;
    std::memcpy(&lutyp, base + c * 168 + 11 * 4, 4);
    std::memcpy(&sltyp, base + c * 168 + 12 * 4, 4);
    const float* zsoil = &w[3];
    const float* zsnow = &w[7];  // snow-layer-top heights, +up
    const int nsnow = (int)std::lround(w[10]);
    const int isn = -nsnow;
    isnow[c] = isn;
    if (static_i) {
      static_i[NMP_I_VEGTYP * ld + c] = lutyp;
      static_i[NMP_I_SOILTYP * ld + c] = sltyp;
    }
    auto S = [&](int f) -> float& { return state[(int64_t)f * ld + c]; };
    S(NMP_S_LAI) = w[13];
    S(NMP_S_SAI) = w[14];
    S(NMP_S_TV) = w[16];
    S(NMP_S_CANLIQ) = w[17];
    S(NMP_S_CANICE) = w[18];
    float snowh = 0.0f;
    for (int j = 0; j < 3; ++j) {
      const bool act = (j - 2) >= isn + 1;
      S(NMP_S_STC + j) = act ? w[19 + j] : 0.0f;    // snowtmp
      S(NMP_S_SNLIQ + j) = act ? w[22 + j] : 0.0f;  // snowwat (mass per area in sflx)
      S(NMP_S_SNICE + j) = act ? w[25 + j] : 0.0f;  // snowice
    }
    // snow layer bottoms from the snow surface: top of layer j is zsnow(j) (+up)
    float top = 0.0f;
    for (int j = 0; j < 3; ++j)
      if ((j - 2) >= isn + 1) top = std::fmax(top, zsnow[j]);
    for (int j = 0; j < 3; ++j) {
      const bool act = (j - 2) >= isn + 1;
      const float bottom = (j < 2 && (j + 1 - 2) >= isn + 1) ? zsnow[j + 1] : 0.0f;
      S(NMP_S_ZSNSO + j) = act ? bottom - top : 0.0f;
    }
    if (isn < 0) snowh = top;
    for (int k = 0; k < 4; ++k) {
      S(NMP_S_STC + 3 + k) = w[28 + k];                  // soiltmp
      S(NMP_S_SH2O + k) = w[32 + k];                     // soilwat
      S(NMP_S_SMC + k) = w[32 + k] + w[36 + k];          // soilwat + soilice
      S(NMP_S_ZSNSO + 3 + k) = zsoil[k] - snowh;         // layer bottoms from snow surface
    }
    S(NMP_S_WA) = w[40];                 // grndwat
    S(NMP_S_ZWT) = -w[41];               // +up -> positive depth
    if (isn < 0) S(NMP_S_SNOWH) = snowh;
  }
  return NMP_OK;
}

}  // extern "C"

namespace {

// One record <-> column c of the SoA host arrays (field f at f*n + c).
template <class T>
struct SflxPack {
  int64_t n;
  std::vector<T> st, sf, fc, dg, fo;
  std::vector<int32_t> isn, si, status;
  explicit SflxPack(int64_t n_)
      : n(n_), st(NMP_NSTATE * n_), sf(NMP_NSTATIC_F * n_), fc(NMP_NFORCING * n_),
        dg(NMP_NDIAG_FULL * n_), fo(NMP_NSNOW * n_), isn(n_), si(NMP_NSTATIC_I * n_),
        status(n_, 0) {}
  T& S(int f, int64_t c) { return st[f * n + c]; }

  void pack(const nmp_sflx_args& r, int64_t c) {
    for (int k = 0; k < NMP_NLAYER; ++k) {
      S(NMP_S_STC + k, c) = r.stc[k];
      S(NMP_S_ZSNSO + k, c) = r.zsnso[k];
    }
    for (int j = 0; j < NMP_NSNOW; ++j) {
      S(NMP_S_SNICE + j, c) = r.snice[j];
      S(NMP_S_SNLIQ + j, c) = r.snliq[j];
      fo[j * n + c] = r.ficeold[j];  // the caller's FICEOLD, as noahmp_sflx takes it
    }
    for (int k = 0; k < NMP_NSOIL; ++k) {
      S(NMP_S_SH2O + k, c) = r.soilwat[k];
      S(NMP_S_SMC + k, c) = r.smc[k];
    }
    const float sc[] = {r.tv,     r.tg,    r.tah,    r.eah,    r.fwet,   r.canliq, r.canice,
                        r.qsfc,   r.snowh, r.sneqv,  r.sneqvo, r.albold, r.tauss,  r.qsnow,
                        r.zwt,    r.wa,    r.wt,     r.wslake, r.lai,    r.sai,    r.lfmass,
                        r.rtmass, r.stmass, r.wood,  r.stblcp, r.fastcp, r.cm,     r.ch};
    for (int i = 0; i < NMP_NSTATE - NMP_S_TV; ++i) S(NMP_S_TV + i, c) = sc[i];
    isn[c] = r.isnow;
    const float f[] = {r.lat, r.zlvl, r.shdfac, r.shdmax, r.tbot, r.foln};
    for (int i = 0; i < NMP_NSTATIC_F; ++i) sf[i * n + c] = f[i];
    const int32_t g[] = {r.lutyp, r.sltyp, r.slptyp, r.isc, r.ist, r.ice};
    for (int i = 0; i < NMP_NSTATIC_I; ++i) si[i * n + c] = g[i];
    const float a[] = {r.sfctmp, r.sfcprs, r.psfc, r.uu,   r.vv,     r.q2,
                       r.soldn,  r.lwdn,   r.prcp, r.cosz, r.co2air, r.o2air};
    for (int i = 0; i < NMP_NFORCING; ++i) fc[i * n + c] = a[i];
  }

  void unpack(nmp_sflx_args& r, int64_t c) {
    for (int k = 0; k < NMP_NLAYER; ++k) {
      r.stc[k] = (float)S(NMP_S_STC + k, c);
      r.zsnso[k] = (float)S(NMP_S_ZSNSO + k, c);
    }
    for (int j = 0; j < NMP_NSNOW; ++j) {
      r.snice[j] = (float)S(NMP_S_SNICE + j, c);
      r.snliq[j] = (float)S(NMP_S_SNLIQ + j, c);
    }
    for (int k = 0; k < NMP_NSOIL; ++k) {
      r.soilwat[k] = (float)S(NMP_S_SH2O + k, c);
      r.smc[k] = (float)S(NMP_S_SMC + k, c);
    }
    float* sc[] = {&r.tv,     &r.tg,     &r.tah,    &r.eah,    &r.fwet,   &r.canliq, &r.canice,
                   &r.qsfc,   &r.snowh,  &r.sneqv,  &r.sneqvo, &r.albold, &r.tauss,  &r.qsnow,
                   &r.zwt,    &r.wa,     &r.wt,     &r.wslake, &r.lai,    &r.sai,    &r.lfmass,
                   &r.rtmass, &r.stmass, &r.wood,   &r.stblcp, &r.fastcp, &r.cm,     &r.ch};
    for (int i = 0; i < NMP_NSTATE - NMP_S_TV; ++i) *sc[i] = (float)S(NMP_S_TV + i, c);
    r.isnow = isn[c];
    for (int d = 0; d < NMP_NDIAG_FULL; ++d) r.out[d] = (float)dg[d * n + c];
    r.status = status[c];
  }
};
static_assert(NMP_NSTATE - NMP_S_TV == 28, "scalar state block");

bool same_f(float a, float b) { return std::memcmp(&a, &b, sizeof(float)) == 0; }

template <class T>
int sflx_columns(nmp_engine* eng, nmp_sflx_args* cols, int64_t n) {
  const nmp_sflx_args& r0 = cols[0];
  for (int64_t c = 0; c < n; ++c) {
    const nmp_sflx_args& r = cols[c];
    if (r.nsoil != NMP_NSOIL || r.nsnow != NMP_NSNOW) return NMP_E_ARG;
    if (r.isnow < -NMP_NSNOW || r.isnow > 0) return NMP_E_ARG;
    if (!same_f(r.dt, r0.dt) || !same_f(r.julian, r0.julian) || r.yearlen != r0.yearlen)
      return NMP_E_ARG;
    if (!julian_ok(r.julian, r.yearlen)) return NMP_E_CALENDAR;
    for (int k = 0; k < NMP_NSOIL; ++k)
      if (!same_f(r.zsoil[k], r0.zsoil[k])) return NMP_E_ARG;
  }
  SflxPack<T> h(n);
  for (int64_t c = 0; c < n; ++c) h.pack(cols[c], c);
  const size_t nb_st = h.st.size() * sizeof(T), nb_sf = h.sf.size() * sizeof(T),
               nb_fc = h.fc.size() * sizeof(T), nb_dg = h.dg.size() * sizeof(T),
               nb_i = (size_t)n * sizeof(int32_t);
  const size_t nb_fo = h.fo.size() * sizeof(T);
  const size_t total = nb_st + nb_sf + nb_fc + nb_dg + nb_fo + nb_i * (2 + NMP_NSTATIC_I);
  char* d = host_scratch(eng, total);
  if (!d) return NMP_E_DEVICE;
  char* p = d;
  auto take = [&](size_t nb) { char* q = p; p += nb; return q; };
  T* d_st = reinterpret_cast<T*>(take(nb_st));
  T* d_sf = reinterpret_cast<T*>(take(nb_sf));
  T* d_fc = reinterpret_cast<T*>(take(nb_fc));
  T* d_dg = reinterpret_cast<T*>(take(nb_dg));
  T* d_fo = reinterpret_cast<T*>(take(nb_fo));
  int32_t* d_isn = reinterpret_cast<int32_t*>(take(nb_i));
  int32_t* d_status = reinterpret_cast<int32_t*>(take(nb_i));
  int32_t* d_si = reinterpret_cast<int32_t*>(take(nb_i * NMP_NSTATIC_I));
  const hipStream_t hs = eng->hstream;
  const auto up = [&](void* dst, const void* src, size_t nb) {
    return hipMemcpyAsync(dst, src, nb, hipMemcpyHostToDevice, hs) == hipSuccess;
  };
  const auto down = [&](void* dst, const void* src, size_t nb) {
    return hipMemcpyAsync(dst, src, nb, hipMemcpyDeviceToHost, hs) == hipSuccess;
  };
  int rc = NMP_OK;
  if (!(up(d_st, h.st.data(), nb_st) && up(d_sf, h.sf.data(), nb_sf) &&
        up(d_fc, h.fc.data(), nb_fc) && up(d_fo, h.fo.data(), nb_fo) &&
        up(d_isn, h.isn.data(), nb_i) && up(d_si, h.si.data(), nb_i * NMP_NSTATIC_I) &&
        hipMemsetAsync(d_status, 0, nb_i, hs) == hipSuccess &&
        hipMemsetAsync(d_dg, 0, nb_dg, hs) == hipSuccess))
    rc = NMP_E_DEVICE;  // (copies already queued are drained below before `h` goes)
  if (rc == NMP_OK)
    rc = launch(eng, n, n, r0.zsoil, r0.dt, r0.julian, r0.yearlen, d_st, d_isn, d_sf, d_si, d_fc,
                d_dg, NMP_DIAG_FULL, d_status, hs, nullptr, nullptr, d_fo);
  if (rc == NMP_OK && !(down(h.st.data(), d_st, nb_st) && down(h.dg.data(), d_dg, nb_dg) &&
                        down(h.isn.data(), d_isn, nb_i) && down(h.status.data(), d_status, nb_i)))
    rc = NMP_E_DEVICE;
  // the copies above may still be in flight (pageable host memory): drain the
  // host stream before the host vectors are read or released
  if (hipStreamSynchronize(hs) != hipSuccess) rc = NMP_E_DEVICE;
  if (rc != NMP_OK) return rc;
  for (int64_t c = 0; c < n; ++c) h.unpack(cols[c], c);
  return NMP_OK;
}

}  // namespace

extern "C" {

int nmp_sflx_columns(nmp_engine* eng, nmp_sflx_args* cols, int64_t n) {
  if (!eng || n < 0 || (n > 0 && !cols)) return NMP_E_ARG;
  if (n == 0) return NMP_OK;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  std::lock_guard<std::mutex> lk(eng->host_mu);
  return eng->precision == 4 ? sflx_columns<float>(eng, cols, n)
                             : sflx_columns<double>(eng, cols, n);
}

int nmp_sflx_column(nmp_engine* eng, nmp_sflx_args* col) { return nmp_sflx_columns(eng, col, 1); }

int nmp_frh2o(nmp_engine* eng, int64_t n, const int32_t* sltyp, const void* tkelv,
              const void* smc, const void* soilwat, void* free_water, int32_t* col_status,
              void* stream) {
  if (!eng || n < 0) return NMP_E_ARG;
  if (n == 0) return NMP_OK;
  if (!sltyp || !tkelv || !smc || !soilwat || !free_water) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return nmp::launch_frh2o(eng->precision, eng->math, eng->dparams, n, sltyp, tkelv, smc, soilwat,
                           free_water, col_status, static_cast<hipStream_t>(stream)) == hipSuccess
             ? NMP_OK
             : NMP_E_DEVICE;
}

int nmp_calhum(nmp_engine* eng, int64_t n, const void* sfctmp, const void* sfcprs, void* q2sat,
               void* dqsdt2, void* stream) {
  if (!eng || n < 0) return NMP_E_ARG;
  if (n == 0) return NMP_OK;
  if (!sfctmp || !sfcprs) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  return nmp::launch_calhum(eng->precision, eng->math, n, sfctmp, sfcprs, q2sat, dqsdt2,
                            static_cast<hipStream_t>(stream)) == hipSuccess
             ? NMP_OK
             : NMP_E_DEVICE;
}

int nmp_frh2o_host(nmp_engine* eng, int64_t n, const int32_t* sltyp, const void* tkelv,
                   const void* smc, const void* soilwat, void* free_water, int32_t* col_status) {
  if (!eng || n < 0) return NMP_E_ARG;
  if (n == 0) return NMP_OK;
  if (!sltyp || !tkelv || !smc || !soilwat || !free_water) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  const size_t nr = (size_t)n * eng->precision, ni = (size_t)n * sizeof(int32_t);
  std::lock_guard<std::mutex> lk(eng->host_mu);
  char* base = host_scratch(eng, 4 * nr + 2 * ni);
  if (!base) return NMP_E_DEVICE;
  char *t = base, *m = t + nr, *w = m + nr, *o = w + nr;
  int32_t* s = reinterpret_cast<int32_t*>(o + nr);
  int32_t* st = s + n;
  const hipStream_t hs = eng->hstream;
  std::vector<int32_t> bits(col_status ? n : 0);
  bool ok = hipMemcpyAsync(t, tkelv, nr, hipMemcpyHostToDevice, hs) == hipSuccess &&
            hipMemcpyAsync(m, smc, nr, hipMemcpyHostToDevice, hs) == hipSuccess &&
            hipMemcpyAsync(w, soilwat, nr, hipMemcpyHostToDevice, hs) == hipSuccess &&
            hipMemcpyAsync(s, sltyp, ni, hipMemcpyHostToDevice, hs) == hipSuccess &&
            hipMemsetAsync(st, 0, ni, hs) == hipSuccess &&
            nmp::launch_frh2o(eng->precision, eng->math, eng->dparams, n, s, t, m, w, o, st, hs) ==
                hipSuccess &&
            hipMemcpyAsync(free_water, o, nr, hipMemcpyDeviceToHost, hs) == hipSuccess &&
            (!col_status ||
             hipMemcpyAsync(bits.data(), st, ni, hipMemcpyDeviceToHost, hs) == hipSuccess);
  if (hipStreamSynchronize(hs) != hipSuccess || !ok) return NMP_E_DEVICE;
  if (col_status)
    for (int64_t i = 0; i < n; ++i) col_status[i] |= bits[i];
  return NMP_OK;
}

int nmp_calhum_host(nmp_engine* eng, int64_t n, const void* sfctmp, const void* sfcprs,
                    void* q2sat, void* dqsdt2) {
  if (!eng || n < 0) return NMP_E_ARG;
  if (n == 0) return NMP_OK;
  if (!sfctmp || !sfcprs) return NMP_E_ARG;
  if (ensure_device(eng->device) != NMP_OK) return NMP_E_DEVICE;
  const size_t nr = (size_t)n * eng->precision;
  std::lock_guard<std::mutex> lk(eng->host_mu);
  char* base = host_scratch(eng, 4 * nr);
  if (!base) return NMP_E_DEVICE;
  char *t = base, *p = t + nr, *q = p + nr, *dq = q + nr;
  const hipStream_t hs = eng->hstream;
  const bool ok =
      hipMemcpyAsync(t, sfctmp, nr, hipMemcpyHostToDevice, hs) == hipSuccess &&
      hipMemcpyAsync(p, sfcprs, nr, hipMemcpyHostToDevice, hs) == hipSuccess &&
      nmp::launch_calhum(eng->precision, eng->math, n, t, p, q2sat ? q : nullptr,
                         dqsdt2 ? dq : nullptr, hs) == hipSuccess &&
      (!q2sat || hipMemcpyAsync(q2sat, q, nr, hipMemcpyDeviceToHost, hs) == hipSuccess) &&
      (!dqsdt2 || hipMemcpyAsync(dqsdt2, dq, nr, hipMemcpyDeviceToHost, hs) == hipSuccess);
  if (hipStreamSynchronize(hs) != hipSuccess || !ok) return NMP_E_DEVICE;
  return NMP_OK;
}

void nmp_finalize(nmp_engine* eng) {
  if (!eng) return;
  ensure_device(eng->device);
  if (eng->hstream) {
    (void)hipStreamSynchronize(eng->hstream);
    (void)hipStreamDestroy(eng->hstream);
  }
  if (eng->scratch) hipFree(eng->scratch);
  if (eng->dparams) hipFree(eng->dparams);
  delete eng;
}

}  // extern "C"
