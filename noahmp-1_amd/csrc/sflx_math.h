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

// Math wrappers are inlined by default; -DNMP_MATH_OUTLINE keeps one copy of
// each (smaller code, fewer instruction-cache misses, call overhead instead).
#ifdef NMP_MATH_OUTLINE
#define NMP_MATH_FN static __device__ __noinline__
#else
#define NMP_MATH_FN static __device__ __forceinline__
#endif

namespace nmp {

template <class T, bool REF>
struct Mth;

template <bool REF>
struct Mth<double, REF> {
  NMP_MATH_FN double exp(double x) { return ::exp(x); }
  NMP_MATH_FN double exp2(double x) { return ::exp2(x); }
  NMP_MATH_FN double log(double x) { return ::log(x); }
  NMP_MATH_FN double log10(double x) { return ::log10(x); }
  NMP_MATH_FN double pow(double x, double y) { return ::pow(x, y); }
  NMP_MATH_FN double tanh(double x) { return ::tanh(x); }
  NMP_MATH_FN double atan(double x) { return ::atan(x); }
  NMP_MATH_FN double tan(double x) { return ::tan(x); }
  NMP_MATH_FN double acos(double x) { return ::acos(x); }
  NMP_MATH_FN double cos(double x) { return ::cos(x); }
  static __device__ __forceinline__ double sqrt(double x) { return ::sqrt(x); }
};

template <>
struct Mth<float, false> {
  NMP_MATH_FN float exp(float x) { return ::expf(x); }
  NMP_MATH_FN float exp2(float x) { return ::exp2f(x); }
  NMP_MATH_FN float log(float x) { return ::logf(x); }
  NMP_MATH_FN float log10(float x) { return ::log10f(x); }
  NMP_MATH_FN float pow(float x, float y) { return ::powf(x, y); }
  NMP_MATH_FN float tanh(float x) { return ::tanhf(x); }
  NMP_MATH_FN float atan(float x) { return ::atanf(x); }
  NMP_MATH_FN float tan(float x) { return ::tanf(x); }
  NMP_MATH_FN float acos(float x) { return ::acosf(x); }
  NMP_MATH_FN float cos(float x) { return ::cosf(x); }
  static __device__ __forceinline__ float sqrt(float x) { return ::sqrtf(x); }
};

template <>
struct Mth<float, true> {
  NMP_MATH_FN float exp(float x) { return (float)::exp((double)x); }
  NMP_MATH_FN float exp2(float x) { return (float)::exp2((double)x); }
  NMP_MATH_FN float log(float x) { return (float)::log((double)x); }
  NMP_MATH_FN float log10(float x) { return (float)::log10((double)x); }
  NMP_MATH_FN float pow(float x, float y) {
    return (float)::pow((double)x, (double)y);
  }
  NMP_MATH_FN float tanh(float x) { return (float)::tanh((double)x); }
  NMP_MATH_FN float atan(float x) { return (float)::atan((double)x); }
  NMP_MATH_FN float tan(float x) { return (float)::tan((double)x); }
  NMP_MATH_FN float acos(float x) { return (float)::acos((double)x); }
  NMP_MATH_FN float cos(float x) { return (float)::cos((double)x); }
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
// The empty asm pins each element as a register value: without it InstCombine
// folds the select chain back into one dynamically indexed load (a[i]), which
// forces the whole enclosing aggregate (the column struct) into scratch.
template <class T>
__device__ __forceinline__ T pin(T v) {
  __asm__ volatile("" : "+v"(v));
  return v;
}
template <class T, int N>
__device__ __forceinline__ T dget(const T (&a)[N], int i) {
  T r = pin(a[0]);
#pragma unroll
  for (int k = 1; k < N; ++k) r = (i == k) ? pin(a[k]) : r;
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
