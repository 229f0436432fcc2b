// Kernel argument block shared by the launch site (engine.hip) and the
// kernel (sflx_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev_params.h"

// workgroup size of the step kernel (256: DESIGN.md "Occupancy")
#ifndef NMP_BLOCK
#define NMP_BLOCK 256
#endif
// per-lane LDS slots for the LDS-resident layer work arrays (LArr)
#ifndef NMP_LDS_SLOTS
#define NMP_LDS_SLOTS 28
#endif

namespace nmp {

struct Opt {
  int veg, crs, btr, run, sfc, frz, inf, rad, alb, snf, tbot, stc;
};

template <class T>
struct KArgs {
  int64_t ncol, ld;
  float zsoil[4];
  float dt, julian;
  int yearlen;
  int diag_level;
  float c_exp_m4, c_albdecay;  // host-precomputed EXP(-4.0), EXP(-0.01*DT/3600) (fp32 ref)
  Opt o;
  T* state;
  int32_t* isnow;
  const T* static_f;
  const int32_t* static_i;
  const T* forcing;
  T* diag;
  int32_t* status;
  // column re-binning (nmp_step_binned): lane i steps column order[i] when
  // order is set; cost (if set) receives each column's loop-cost key
  const int32_t* order;
  uint8_t* cost;
  // noahmp_sflx's FICEOLD argument (3 x ld), or NULL: derived from
  // SNICE/SNLIQ at step start (offline-driver convention)
  const T* ficeold;
  // columns stepped per 64-lane wave (8..64, a multiple of 8): below 64 the
  // launch spreads a small column set over more waves (small-N latency hiding)
  int cpw;
#ifdef NMP_TRUNC_RUNTIME
  int trunc_at;  // (probe builds) phase mark the step returns at (sflx_kernel.hip)
#endif
};

template <class T, bool R>
hipError_t launch_sflx(const DevParams* dparams, const KArgs<T>& a, hipStream_t stream,
                       bool small, int os);

// csrc/forcing.hip: synthetic forcing of one step from the climate records
hipError_t launch_forcing_synth(int precision, int64_t ncol, int64_t ld, const void* clim,
                                double julian, int32_t yearlen, uint64_t seed, int64_t step,
                                int64_t first_col, void* out, hipStream_t stream);

// csrc/forcing.hip: the 12 forcing fields from the LDASIN block (fp32); with
// geo (not null) COSZ formed on the device from the columns' geometry
hipError_t launch_forcing_ldasin(int precision, int64_t ncol, int64_t ld, const float* in,
                                 const double* geo, double sin_decl, double cos_decl, double ha0,
                                 void* out, hipStream_t stream);
// csrc/forcing.hip: an LDASIN file's big-endian grids -> the block's 8 rows
hipError_t launch_ldasin_ingest(int64_t ncol, int64_t ld, int64_t npts, const void* grid_be,
                                const int32_t* point, float* block, hipStream_t stream);
// csrc/forcing.hip: diagnostics -> the LDASOUT file's big-endian grids
hipError_t launch_ldasout_grid(int precision, int64_t ncol, int64_t ld, int64_t npts, int nfield,
                               const void* diag, const int32_t* point, double fill, void* grid_be,
                               hipStream_t stream);

// csrc/routines.hip: the reference's public routines frh2o / calhum over n
// elements (device pointers, engine precision; math 0 = the fp32 "ref" policy)
hipError_t launch_frh2o(int precision, int math, const DevParams* P, int64_t n,
                        const int32_t* sltyp, const void* tkelv, const void* smc, const void* sh2o,
                        void* out, int32_t* status, hipStream_t stream);
hipError_t launch_calhum(int precision, int math, int64_t n, const void* sfctmp,
                         const void* sfcprs, void* q2sat, void* dqsdt2, hipStream_t stream);

// csrc/rebin.hip: per-tile counting sort of the columns by cost key
hipError_t launch_rebin(const uint8_t* cost, int32_t* order, int64_t ncol, int tile,
                        hipStream_t stream);

}  // namespace nmp
