// The reference's public physics routines besides noahmp_sflx, as batched
// device launches behind the C ABI (include/noahmp_engine.h nmp_frh2o /
// nmp_calhum):
//   frh2o   func.f90:4494-4598   (public: func.f90:6-8)
//   calhum  func.f90:3958-3984   (module procedure, public by default)
// Each lane evaluates the SAME device routine the step kernel inlines
// (csrc/sflx_routines.h), so a Fortran caller of `frh2o` / `calhum` gets the
// values noahmp_sflx computes internally: bit-identical to the reference in
// the fp32 "ref" math policy (tests/test_gpu_routines.py).
#include <hip/hip_runtime.h>

#include "sflx_routines.h"

namespace nmp {
namespace {

constexpr int kBlock = 256;

// frh2o's soil parameters come from the engine's tables (LK_BEXP, LK_PSISAT,
// LK_SMCMAX of the soil type, as the reference's module arrays: rows past the
// table's soil types are NaN there and here); a soil type outside the arrays
// yields NaN and NMP_ST_STOP instead of an out-of-range read.
template <class T, bool R>
__global__ __launch_bounds__(kBlock) void frh2o_kernel(const DevParams* __restrict__ P, int64_t n,
                                                       const int32_t* __restrict__ sltyp,
                                                       const T* __restrict__ tkelv,
                                                       const T* __restrict__ smc,
                                                       const T* __restrict__ sh2o,
                                                       T* __restrict__ out,
                                                       int32_t* __restrict__ status) {
  if constexpr (sizeof(T) == 4 && R) {
    stage_math_tables();
    __syncthreads();
  }
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int st = sltyp[i];
  int bits = 0;
  T v;
  if (st < 1 || st > NMP_MSLTYP) {
    v = (T)NAN;
    bits = NMP_ST_STOP;
  } else {
    const SoilRec& S = P->soil[st - 1];
    v = frh2o<T, R>((T)S.smcmax, (T)S.psisat, (T)S.bexp, tkelv[i], smc[i], sh2o[i], bits);
  }
  out[i] = v;
  if (status && bits) status[i] |= bits;
}

template <class T, bool R>
__global__ __launch_bounds__(kBlock) void calhum_kernel(int64_t n, const T* __restrict__ sfctmp,
                                                        const T* __restrict__ sfcprs,
                                                        T* __restrict__ q2sat,
                                                        T* __restrict__ dqsdt2) {
  if constexpr (sizeof(T) == 4 && R) {
    stage_math_tables();
    __syncthreads();
  }
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  T q, d;
  calhum<T, R>(sfctmp[i], sfcprs[i], q, d);
  if (q2sat) q2sat[i] = q;
  if (dqsdt2) dqsdt2[i] = d;
}

dim3 grid_for(int64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

}  // namespace

hipError_t launch_frh2o(int precision, int math, const DevParams* P, int64_t n,
                        const int32_t* sltyp, const void* tkelv, const void* smc, const void* sh2o,
                        void* out, int32_t* status, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (precision == 4) {
    auto k = math == 0 ? frh2o_kernel<float, true> : frh2o_kernel<float, false>;
    hipLaunchKernelGGL(k, grid_for(n), dim3(kBlock), 0, stream, P, n, sltyp,
                       static_cast<const float*>(tkelv), static_cast<const float*>(smc),
                       static_cast<const float*>(sh2o), static_cast<float*>(out), status);
  } else {
    hipLaunchKernelGGL((frh2o_kernel<double, false>), grid_for(n), dim3(kBlock), 0, stream, P, n,
                       sltyp, static_cast<const double*>(tkelv), static_cast<const double*>(smc),
                       static_cast<const double*>(sh2o), static_cast<double*>(out), status);
  }
  return hipGetLastError();
}

hipError_t launch_calhum(int precision, int math, int64_t n, const void* sfctmp,
                         const void* sfcprs, void* q2sat, void* dqsdt2, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (precision == 4) {
    auto k = math == 0 ? calhum_kernel<float, true> : calhum_kernel<float, false>;
    hipLaunchKernelGGL(k, grid_for(n), dim3(kBlock), 0, stream, n,
                       static_cast<const float*>(sfctmp), static_cast<const float*>(sfcprs),
                       static_cast<float*>(q2sat), static_cast<float*>(dqsdt2));
  } else {
    hipLaunchKernelGGL((calhum_kernel<double, false>), grid_for(n), dim3(kBlock), 0, stream, n,
                       static_cast<const double*>(sfctmp), static_cast<const double*>(sfcprs),
                       static_cast<double*>(q2sat), static_cast<double*>(dqsdt2));
  }
  return hipGetLastError();
}

}  // namespace nmp
