// Synthetic LDASIN-style forcing generated on the device (SURVEY.md 8d,
// config #5: "forcing generated on device from a counter-based hash"; a year of
// hourly forcing for 1 M columns streamed from the host would be 0.4-0.8 TB).
//
// The reference reads forcing from LDASIN files (run/case.nml:6-7) and ships
// none, so the synthetic cases (noahmp-1_amd/cases.py) define their own
// diurnal climate per column.  This kernel is that generator with its random
// draws taken from a stateless counter-based hash of (seed, step, column,
// draw): any step of any column can be produced independently, on any rank,
// in any order, with no generator state to carry or shard.  Every value is
// computed in double and rounded once to the engine precision; the numpy
// restatement in tests/test_gpu_forcing.py follows it operation for operation.
//
// Per column, field-major (ld apart): the climate record NMP_CLIM_* (lat and
// lon in radians, mean temperature, diurnal amplitude, relative humidity,
// pressure, mean wind u/v, precipitation probability); out: the 12 NMP_A_*
// forcing fields of one step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "noahmp_engine.h"

namespace nmp {

__device__ __forceinline__ uint64_t mix64(uint64_t h) {
  h ^= h >> 30;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 27;
  h *= 0x94D049BB133111EBull;
  h ^= h >> 31;
  return h;
}

// uniform in [0, 1): 53 hash bits
__device__ __forceinline__ double uhash(uint64_t key, uint64_t draw) {
  return (double)(mix64(key + draw * 0xF1357AEA2E62A9C5ull) >> 11) * 0x1.0p-53;
}

// standard normal (Box-Muller on draws d, d+1; 1 - u keeps the log finite)
__device__ __forceinline__ double nhash(uint64_t key, uint64_t d) {
  const double u1 = 1.0 - uhash(key, d), u2 = uhash(key, d + 1);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

template <class T>
__global__ __launch_bounds__(256) void forcing_synth_kernel(int64_t ncol, int64_t ld,
                                                            const T* __restrict__ clim,
                                                            double julian, int32_t yearlen,
                                                            uint64_t seed, int64_t step,
                                                            int64_t first_col,
                                                            T* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncol) return;
  const double lat = (double)clim[NMP_CLIM_LAT * ld + c];
  const double lon = (double)clim[NMP_CLIM_LON * ld + c];
  const double t0 = (double)clim[NMP_CLIM_T0 * ld + c];
  const double amp = (double)clim[NMP_CLIM_AMP * ld + c];
  const double rh = (double)clim[NMP_CLIM_RH * ld + c];
  const double pres = (double)clim[NMP_CLIM_PRES * ld + c];
  const double wu = (double)clim[NMP_CLIM_WIND_U * ld + c];
  const double wv = (double)clim[NMP_CLIM_WIND_V * ld + c];
  const double wet = (double)clim[NMP_CLIM_WET * ld + c];
  const uint64_t key = seed * 0x9E3779B97F4A7C15ull + (uint64_t)step * 0xD1B54A32D192ED03ull +
                       (uint64_t)(first_col + c) * 0xAEF17502108EF2D9ull;
  const double pi = 3.141592653589793;
  // diurnal temperature at local solar time (cases.forcing_step)
  const double frac = julian - floor(julian);
  const double hour = fmod(frac * 24.0 + lon * (180.0 / pi) / 15.0 + 48.0, 24.0);
  const double t = t0 + amp * cos(2.0 * pi * (hour - 14.0) / 24.0) + 0.3 * nhash(key, 0);
  // solar geometry (timeman.cosz)
  const double decl = 0.409 * sin(2.0 * pi * (julian - 80.0) / (double)yearlen);
  const double ha = 2.0 * pi * frac + lon - pi;
  const double cz = sin(lat) * sin(decl) + cos(lat) * cos(decl) * cos(ha);
  const double cloud = 0.6 * uhash(key, 2);
  const double soldn = (cz > 0.0 ? cz : 0.0) * 1000.0 * (1.0 - 0.6 * cloud);
  const double lwdn = (0.72 + 0.2 * cloud) * 5.67e-8 * (t * t) * (t * t);
  const double e = rh * 611.2 * exp(17.67 * (t - 273.15) / (t - 29.65));
  const double q2 = 0.622 * e / (pres - 0.378 * e);
  const double prcp = uhash(key, 3) < wet ? -1.0e-3 * log(1.0 - uhash(key, 4)) : 0.0;
  T* o = out + c;
  o[NMP_A_SFCTMP * ld] = (T)t;
  o[NMP_A_SFCPRS * ld] = (T)pres;
  o[NMP_A_PSFC * ld] = (T)pres;
  o[NMP_A_UU * ld] = (T)(wu + 0.7 * nhash(key, 5));
  o[NMP_A_VV * ld] = (T)(wv + 0.7 * nhash(key, 7));
  o[NMP_A_Q2 * ld] = (T)q2;
  o[NMP_A_SOLDN * ld] = (T)soldn;
  o[NMP_A_LWDN * ld] = (T)lwdn;
  o[NMP_A_PRCP * ld] = (T)prcp;
  o[NMP_A_COSZ * ld] = (T)cz;
  o[NMP_A_CO2AIR * ld] = (T)(395.0e-6 * pres);
  o[NMP_A_O2AIR * ld] = (T)(0.209 * pres);
}

hipError_t launch_forcing_synth(int precision, int64_t ncol, int64_t ld, const void* clim,
                                double julian, int32_t yearlen, uint64_t seed, int64_t step,
                                int64_t first_col, void* out, hipStream_t stream) {
  const int64_t grid = (ncol + 255) / 256;
  if (grid == 0) return hipSuccess;
  if (precision == 4)
    hipLaunchKernelGGL(forcing_synth_kernel<float>, dim3((unsigned)grid), dim3(256), 0, stream,
                       ncol, ld, static_cast<const float*>(clim), julian, yearlen, seed, step,
                       first_col, static_cast<float*>(out));
  else
    hipLaunchKernelGGL(forcing_synth_kernel<double>, dim3((unsigned)grid), dim3(256), 0, stream,
                       ncol, ld, static_cast<const double*>(clim), julian, yearlen, seed, step,
                       first_col, static_cast<double*>(out));
  return hipGetLastError();
}

// LDASIN forcing as the files carry it -> the 12 noahmp_sflx forcing fields
// (nmp_forcing_from_ldasin).  The host uploads the 8 LDASIN variables plus
// COSZ in fp32 (36 B per column instead of 48, or 96 for an fp64 engine) and
// the fields noahmp_sflx takes twice or derives are formed here exactly as
// the host reader forms them (noahmp-1_amd/ncio.py LdasinForcing):
// SFCPRS = PSFC = the file's PSFC, CO2AIR = 395e-6 PSFC and O2AIR = 0.209 PSFC
// as one IEEE double product of the fp32 pressure rounded once to fp32, every
// field then widened to the engine precision (the host's fp32 array uploaded
// into a T buffer).
//
// GEO (nmp_forcing_from_ldasin_geo): COSZ is not read from the block but
// formed per column from its latitude factors and longitude (geo, (3, ld)
// double: sin lat, cos lat, lon) and the step's solar terms, with
// timeman.cosz's expression and operation order in double --
// sin_lat sin_decl + (cos_lat cos_decl) cos((ha0 + lon) - pi) -- rounded once
// to fp32.  The block's 8 file variables then stay resident on the device for
// every step of their input interval: nothing is uploaded between files.
template <class T, bool GEO>
__global__ __launch_bounds__(256) void forcing_ldasin_kernel(int64_t ncol, int64_t ld,
                                                             const float* __restrict__ in,
                                                             const double* __restrict__ geo,
                                                             double sin_decl, double cos_decl,
                                                             double ha0, T* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncol) return;
  const float* i = in + c;
  const float psfc = i[NMP_L_PSFC * ld];
  float cosz;
  if constexpr (GEO) {
    const double* g = geo + c;
    const double ha = (ha0 + g[2 * ld]) - 3.141592653589793;
    cosz = (float)(g[0] * sin_decl + (g[ld] * cos_decl) * cos(ha));
  } else {
    cosz = i[NMP_L_COSZ * ld];
  }
  T* o = out + c;
  o[NMP_A_SFCTMP * ld] = (T)i[NMP_L_T2D * ld];
  o[NMP_A_SFCPRS * ld] = (T)psfc;
  o[NMP_A_PSFC * ld] = (T)psfc;
  o[NMP_A_UU * ld] = (T)i[NMP_L_U2D * ld];
  o[NMP_A_VV * ld] = (T)i[NMP_L_V2D * ld];
  o[NMP_A_Q2 * ld] = (T)i[NMP_L_Q2D * ld];
  o[NMP_A_SOLDN * ld] = (T)i[NMP_L_SWDOWN * ld];
  o[NMP_A_LWDN * ld] = (T)i[NMP_L_LWDOWN * ld];
  o[NMP_A_PRCP * ld] = (T)i[NMP_L_RAINRATE * ld];
  o[NMP_A_COSZ * ld] = (T)cosz;
  o[NMP_A_CO2AIR * ld] = (T)(float)(395.0e-6 * (double)psfc);
  o[NMP_A_O2AIR * ld] = (T)(float)(0.209 * (double)psfc);
}

template <class T>
static void launch_ldasin_t(int64_t grid, int64_t ncol, int64_t ld, const float* in,
                            const double* geo, double sd, double cd, double ha0, T* out,
                            hipStream_t stream) {
  if (geo)
    hipLaunchKernelGGL((forcing_ldasin_kernel<T, true>), dim3((unsigned)grid), dim3(256), 0,
                       stream, ncol, ld, in, geo, sd, cd, ha0, out);
  else
    hipLaunchKernelGGL((forcing_ldasin_kernel<T, false>), dim3((unsigned)grid), dim3(256), 0,
                       stream, ncol, ld, in, geo, sd, cd, ha0, out);
}

hipError_t launch_forcing_ldasin(int precision, int64_t ncol, int64_t ld, const float* in,
                                 const double* geo, double sin_decl, double cos_decl, double ha0,
                                 void* out, hipStream_t stream) {
  const int64_t grid = (ncol + 255) / 256;
  if (grid == 0) return hipSuccess;
  if (precision == 4)
    launch_ldasin_t(grid, ncol, ld, in, geo, sin_decl, cos_decl, ha0, static_cast<float*>(out),
                    stream);
  else
    launch_ldasin_t(grid, ncol, ld, in, geo, sin_decl, cos_decl, ha0, static_cast<double*>(out),
                    stream);
  return hipGetLastError();
}

// An LDASIN file's 8 variables as the netCDF-3 file stores them -- each a
// big-endian fp32 grid of npts points, in NMP_L_* order -- into the block's
// rows NMP_L_T2D..NMP_L_LWDOWN in engine column order (nmp_ldasin_ingest):
// column c takes grid point point[c].  The host only copies the file's bytes;
// the land-point selection, the engine's column order and the byte order are
// applied here, one gathered 4-byte load per variable and column.
__global__ __launch_bounds__(256) void ldasin_ingest_kernel(int64_t ncol, int64_t ld, int64_t npts,
                                                            const uint32_t* __restrict__ grid_be,
                                                            const int32_t* __restrict__ point,
                                                            float* __restrict__ block) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncol) return;
  const int64_t p = point[c];
  if (p < 0 || p >= npts) {  // outside the grid: NaN, never an out-of-bounds load
#pragma unroll
    for (int v = 0; v < NMP_L_COSZ; ++v) block[v * ld + c] = __int_as_float(0x7fc00000);
    return;
  }
#pragma unroll
  for (int v = 0; v < NMP_L_COSZ; ++v)
    block[v * ld + c] = __uint_as_float(__builtin_bswap32(grid_be[v * npts + p]));
}

hipError_t launch_ldasin_ingest(int64_t ncol, int64_t ld, int64_t npts, const void* grid_be,
                                const int32_t* point, float* block, hipStream_t stream) {
  const int64_t grid = (ncol + 255) / 256;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(ldasin_ingest_kernel, dim3((unsigned)grid), dim3(256), 0, stream, ncol, ld,
                     npts, static_cast<const uint32_t*>(grid_be), point, block);
  return hipGetLastError();
}

// The output side's mirror (nmp_ldasout_grid): nfield diagnostics of ncol
// columns (engine precision T, field-major, leading dimension ld) onto the
// file's grids as a netCDF-3 file stores them -- big-endian T, npts points
// per field, `fill` where no column lands -- so the host writes the bytes
// as they are.  One pass fills the grids, a second scatters the columns.
template <class T, class W>
__global__ __launch_bounds__(256) void grid_fill_kernel(int64_t total, W fill_be,
                                                        W* __restrict__ grid_be) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x)
    grid_be[i] = fill_be;
}

template <class T, class W>
__global__ __launch_bounds__(256) void grid_scatter_kernel(int64_t ncol, int64_t ld, int64_t npts,
                                                           int nfield, const W* __restrict__ diag,
                                                           const int32_t* __restrict__ point,
                                                           W* __restrict__ grid_be) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncol) return;
  const int64_t p = point[c];
  if (p < 0 || p >= npts) return;  // outside the grid: never an out-of-bounds store
  for (int f = 0; f < nfield; ++f) {
    const W w = diag[f * ld + c];
    if constexpr (sizeof(W) == 4)
      grid_be[f * npts + p] = __builtin_bswap32(w);
    else
      grid_be[f * npts + p] = __builtin_bswap64(w);
  }
}

template <class T, class W>
static hipError_t launch_grid_t(int64_t ncol, int64_t ld, int64_t npts, int nfield,
                                const void* diag, const int32_t* point, double fill,
                                void* grid_be, hipStream_t stream) {
  const T f = (T)fill;
  W fw;
  __builtin_memcpy(&fw, &f, sizeof(W));
  if constexpr (sizeof(W) == 4)
    fw = __builtin_bswap32(fw);
  else
    fw = __builtin_bswap64(fw);
  const int64_t total = (int64_t)nfield * npts;
  const int64_t fgrid = std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL((grid_fill_kernel<T, W>), dim3((unsigned)fgrid), dim3(256), 0, stream, total,
                     fw, static_cast<W*>(grid_be));
  const int64_t grid = (ncol + 255) / 256;
  if (grid > 0)
    hipLaunchKernelGGL((grid_scatter_kernel<T, W>), dim3((unsigned)grid), dim3(256), 0, stream,
                       ncol, ld, npts, nfield, static_cast<const W*>(diag), point,
                       static_cast<W*>(grid_be));
  return hipGetLastError();
}

hipError_t launch_ldasout_grid(int precision, int64_t ncol, int64_t ld, int64_t npts, int nfield,
                               const void* diag, const int32_t* point, double fill, void* grid_be,
                               hipStream_t stream) {
  if (npts == 0 || nfield == 0) return hipSuccess;
  if (precision == 4)
    return launch_grid_t<float, uint32_t>(ncol, ld, npts, nfield, diag, point, fill, grid_be,
                                          stream);
  return launch_grid_t<double, uint64_t>(ncol, ld, npts, nfield, diag, point, fill, grid_be,
                                         stream);
}

}  // namespace nmp
