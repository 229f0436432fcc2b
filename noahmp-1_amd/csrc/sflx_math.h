// Arithmetic helpers for the sflx kernel (device side).
//
// Transcendental policy:
//  - Mth<float, true>  "ref":  float functions evaluated in double and rounded once to
//    float.  glibc's float functions used by the reference (compiled by
//    amdflang, core/module_noahmp_func.f90) are correctly rounded or within
//    ~0.5-0.8 ulp, so this policy reproduces their results in all but rare
//    near-midpoint cases.  Parity mode.
//  - Mth<float, false> "fast": ocml single-precision functions (<= ~1-2 ulp).
//  - Mth<double, *>:          ocml double functions (fp64 engine).
// Division and sqrt are IEEE correctly rounded in every policy (hipcc default
// -fhip-fp32-correctly-rounded-divide-sqrt), and the kernel is compiled with
// -ffp-contract=off so products and sums round exactly like the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace nmp {

template <class T, bool REF>
struct Mth;

template <bool REF>
struct Mth<double, REF> {
  static __device__ __forceinline__ double exp(double x) { return ::exp(x); }
  static __device__ __forceinline__ double exp2(double x) { return ::exp2(x); }
  static __device__ __forceinline__ double log(double x) { return ::log(x); }
  static __device__ __forceinline__ double log10(double x) { return ::log10(x); }
  static __device__ __forceinline__ double pow(double x, double y) { return ::pow(x, y); }
  static __device__ __forceinline__ double tanh(double x) { return ::tanh(x); }
  static __device__ __forceinline__ double atan(double x) { return ::atan(x); }
  static __device__ __forceinline__ double tan(double x) { return ::tan(x); }
  static __device__ __forceinline__ double acos(double x) { return ::acos(x); }
  static __device__ __forceinline__ double cos(double x) { return ::cos(x); }
  static __device__ __forceinline__ double sqrt(double x) { return ::sqrt(x); }
};

template <>
struct Mth<float, false> {
  static __device__ __forceinline__ float exp(float x) { return ::expf(x); }
  static __device__ __forceinline__ float exp2(float x) { return ::exp2f(x); }
  static __device__ __forceinline__ float log(float x) { return ::logf(x); }
  static __device__ __forceinline__ float log10(float x) { return ::log10f(x); }
  static __device__ __forceinline__ float pow(float x, float y) { return ::powf(x, y); }
  static __device__ __forceinline__ float tanh(float x) { return ::tanhf(x); }
  static __device__ __forceinline__ float atan(float x) { return ::atanf(x); }
  static __device__ __forceinline__ float tan(float x) { return ::tanf(x); }
  static __device__ __forceinline__ float acos(float x) { return ::acosf(x); }
  static __device__ __forceinline__ float cos(float x) { return ::cosf(x); }
  static __device__ __forceinline__ float sqrt(float x) { return ::sqrtf(x); }
};

template <>
struct Mth<float, true> {
  static __device__ __forceinline__ float exp(float x) { return (float)::exp((double)x); }
  static __device__ __forceinline__ float exp2(float x) { return (float)::exp2((double)x); }
  static __device__ __forceinline__ float log(float x) { return (float)::log((double)x); }
  static __device__ __forceinline__ float log10(float x) { return (float)::log10((double)x); }
  static __device__ __forceinline__ float pow(float x, float y) {
    return (float)::pow((double)x, (double)y);
  }
  static __device__ __forceinline__ float tanh(float x) { return (float)::tanh((double)x); }
  static __device__ __forceinline__ float atan(float x) { return (float)::atan((double)x); }
  static __device__ __forceinline__ float tan(float x) { return (float)::tan((double)x); }
  static __device__ __forceinline__ float acos(float x) { return (float)::acos((double)x); }
  static __device__ __forceinline__ float cos(float x) { return (float)::cos((double)x); }
  static __device__ __forceinline__ float sqrt(float x) { return ::sqrtf(x); }
};

template <class T>
__device__ __forceinline__ T rmax(T a, T b) { return a > b ? a : b; }
template <class T>
__device__ __forceinline__ T rmin(T a, T b) { return a < b ? a : b; }
// integer powers as the reference's compiler lowers them: sequential products
template <class T>
__device__ __forceinline__ T p2(T x) { return x * x; }
template <class T>
__device__ __forceinline__ T p3(T x) { return x * (x * x); }
template <class T>
__device__ __forceinline__ T p4(T x) { return x * p3(x); }
template <class T>
__device__ __forceinline__ T p5(T x) { return x * p4(x); }

// Register-array access with a runtime index, lowered to a select chain so the
// array itself stays in VGPRs (a dynamic subscript would demote it to scratch).
template <class T, int N>
__device__ __forceinline__ T dget(const T (&a)[N], int i) {
  T r = a[0];
#pragma unroll
  for (int k = 1; k < N; ++k) r = (i == k) ? a[k] : r;
  return r;
}
template <class T, int N>
__device__ __forceinline__ void dset(T (&a)[N], int i, T v) {
#pragma unroll
  for (int k = 0; k < N; ++k)
    if (i == k) a[k] = v;
}
__device__ __forceinline__ float zget(const float (&a)[4], int i) {
  return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

}  // namespace nmp

// literal in the working precision: fp32 literals are parsed as float (like the
// reference's default-real constants), fp64 literals as double
#define L(x) (sizeof(T) == 4 ? (T)(x##f) : (T)(x))
