// Arithmetic helpers for the sflx kernel (device side).
//
// Transcendental policy:
//  - Mth<float, true>  "ref":  bit-exact restatements of the glibc 2.35 float
//    libm the reference's compiled physics calls (glibc_math.h: expf, exp2f,
//    logf, powf, tanhf, atanf, log10f, acosf, cosf, tanf).  Each is checked
//    against the host libm over all 2^32 inputs (powf: 26e9 samples), so the
//    kernel's elementary functions return exactly what the reference's do.
//    Their small tables (768 B) are staged per workgroup in LDS.  Default.
//  - Mth<float, false> "fast": ocml single-precision functions (<= ~1-2 ulp).
//  - Mth<double, *>:          ocml double functions (fp64 engine).
// Division and sqrt are IEEE correctly rounded in every policy (hipcc default
// -fhip-fp32-correctly-rounded-divide-sqrt), and the kernel is compiled with
// -ffp-contract=off so products and sums round exactly like the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "glibc_math.h"

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

// fp64 exp with a short dependent chain (NMP_F64_EXP_ESTRIN): ocml's own
// reduction (k = rint(x/ln2), r = x - k ln2 in two parts) and its degree-11
// Taylor coefficients, but the polynomial evaluated by Estrin's scheme (depth
// 4 instead of 11 dependent FMAs) and rebuilt with ldexp.  The fp64 path is
// held to tolerances, not bits (DESIGN.md "fp64"); the result is within an ulp
// or two of ocml's.  Aimed at config #2, whose one wave per SIMD runs every
// dependent chain at full latency.
#ifndef NMP_F64_EXP_ESTRIN
#define NMP_F64_EXP_ESTRIN 0
#endif
__device__ __forceinline__ double exp_estrin(double x) {
  const double k = __builtin_rint(x * 1.4426950408889634);     // x / ln2
  double r = __builtin_fma(k, -0.6931471805599453, x);          // ln2, then its tail
  r = __builtin_fma(k, -2.3190468138462996e-17, r);
  const double r2 = r * r, r4 = r2 * r2, r8 = r4 * r4;
  // ocml's coefficients c0..c11 (c0 = c1 = 1), paired by Estrin's scheme
  const double q0 = __builtin_fma(r, 1.0, 1.0);
  const double q1 = __builtin_fma(r, 0.16666666666666477, 0.5000000000000012);
  const double q2 = __builtin_fma(r, 0.008333333333455043, 0.041666666666519754);
  const double q3 = __builtin_fma(r, 0.00019841269589115522, 0.0013888888945916382);
  const double q4 = __builtin_fma(r, 2.755751454582531e-06, 2.480149103909504e-05);
  const double q5 = __builtin_fma(r, 2.502232256764614e-08, 2.7630903490112654e-07);
  const double s0 = __builtin_fma(r2, q1, q0);
  const double s1 = __builtin_fma(r2, q3, q2);
  const double s2 = __builtin_fma(r2, q5, q4);
  const double p = __builtin_fma(r8, s2, __builtin_fma(r4, s1, s0));
  const double e = __builtin_ldexp(p, (int)k);
  // ocml's limits: +inf above 1024, 0 below -1075 (ldexp saturates between);
  // NaN propagates through r
  return x > 1024.0 ? __builtin_inf() : (x < -1075.0 ? 0.0 : e);
}

template <bool REF>
struct Mth<double, REF> {
#if NMP_F64_EXP_ESTRIN
  NMP_MATH_FN double exp(double x) { return exp_estrin(x); }
#else
  NMP_MATH_FN double exp(double x) { return ::exp(x); }
#endif
  NMP_MATH_FN double exp2(double x) { return ::exp2(x); }
  NMP_MATH_FN double log(double x) { return ::log(x); }
  NMP_MATH_FN double log10(double x) { return ::log10(x); }
#ifdef NMP_F64_OCML_POW
  NMP_MATH_FN double pow(double x, double y) { return ::pow(x, y); }
#else
  // x**y as exp(y log x): within |y log x| ulp of pow, which is far inside the
  // fp64 path's tolerances, at about half the cost of ocml's double pow (that
  // one carries log x in double-double).  Every base in the kernel is >= 0;
  // 0**y (y > 0) -> exp(-inf) = 0 as pow gives.
  NMP_MATH_FN double pow(double x, double y) { return exp(y * ::log(x)); }
#endif
  // x**0.25 and x**(-0.25): the fp64 path is held to a tolerance, not to bits
  // (DESIGN.md "fp64"), so the fourth root is two square roots (<= 1 ulp from
  // pow, and ~10x cheaper than ocml's double pow)
  NMP_MATH_FN double pow_q(double x) { return ::sqrt(::sqrt(x)); }
  NMP_MATH_FN double pow_mq(double x) { return 1.0 / ::sqrt(::sqrt(x)); }
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
  NMP_MATH_FN float pow_q(float x) { return ::powf(x, 0.25f); }
  NMP_MATH_FN float pow_mq(float x) { return ::powf(x, -0.25f); }
  NMP_MATH_FN float tanh(float x) { return ::tanhf(x); }
  NMP_MATH_FN float atan(float x) { return ::atanf(x); }
  NMP_MATH_FN float tan(float x) { return ::tanf(x); }
  NMP_MATH_FN float acos(float x) { return ::acosf(x); }
  NMP_MATH_FN float cos(float x) { return ::cosf(x); }
  static __device__ __forceinline__ float sqrt(float x) { return ::sqrtf(x); }
};

// glibc libm tables: one __constant__ master copy, staged into LDS by every
// workgroup's prologue (stage_math_tables) before first use.
static __shared__ gm::GmTables gm_lds;
static __constant__ gm::GmTables gm_const = {GM_EXP2F_TAB, GM_LOGF_TAB, GM_POWF_TAB};

// NMP_PARAMS_GLOBAL (probe builds): the tables are read from global memory
// (L1/L2-resident) instead of being staged per workgroup into LDS
#ifdef NMP_PARAMS_GLOBAL
#define NMP_GM_TAB gm_const
#else
#define NMP_GM_TAB gm_lds
#endif
__device__ __forceinline__ void stage_math_tables() {
  constexpr int NW = sizeof(gm::GmTables) / sizeof(int4);
  static_assert(sizeof(gm::GmTables) % sizeof(int4) == 0, "table size");
  const int4* src = reinterpret_cast<const int4*>(&gm_const);
  int4* dst = reinterpret_cast<int4*>(&gm_lds);
  for (int i = threadIdx.x; i < NW; i += blockDim.x) dst[i] = src[i];
}

template <>
struct Mth<float, true> {
  NMP_MATH_FN float exp(float x) { return gm::expf(x, NMP_GM_TAB); }
  NMP_MATH_FN float exp2(float x) { return gm::exp2f(x, NMP_GM_TAB); }
  NMP_MATH_FN float log(float x) { return gm::logf(x, NMP_GM_TAB); }
  NMP_MATH_FN float log10(float x) { return gm::log10f(x, NMP_GM_TAB); }
  NMP_MATH_FN float pow(float x, float y) { return gm::powf(x, y, NMP_GM_TAB); }
  // bit-exact fp32: the reference's powf itself
  NMP_MATH_FN float pow_q(float x) { return gm::powf(x, 0.25f, NMP_GM_TAB); }
  NMP_MATH_FN float pow_mq(float x) { return gm::powf(x, -0.25f, NMP_GM_TAB); }
  NMP_MATH_FN float tanh(float x) { return gm::tanhf(x); }
  NMP_MATH_FN float atan(float x) { return gm::atanf(x); }
  NMP_MATH_FN float tan(float x) { return gm::tanf(x); }
  NMP_MATH_FN float acos(float x) { return gm::acosf(x); }
  NMP_MATH_FN float cos(float x) { return gm::cosf(x); }
  static __device__ __forceinline__ float sqrt(float x) { return ::sqrtf(x); }
};

// x**y1 and x**y2 with one base (wdfcnd1/wdfcnd2's WDF and WCND): each equal
// to Mth::pow's result bit for bit.  The fp32 "ref" path forms powf's log2 of
// x once (gm::powf_pair); the fp64 path (exp(y log x)) its log once.
// NMP_POW_PAIR=0: two independent calls (A/B probe).
#ifndef NMP_POW_PAIR
#define NMP_POW_PAIR 1
#endif
template <class T, bool R>
__device__ __forceinline__ void pow_pair(T x, T y1, T y2, T& r1, T& r2) {
#if NMP_POW_PAIR
  if constexpr (sizeof(T) == 4 && R) {
    gm::powf_pair(x, y1, y2, NMP_GM_TAB, r1, r2);
    return;
  }
#ifndef NMP_F64_OCML_POW
  if constexpr (sizeof(T) == 8) {
    const double lx = ::log(x);
    r1 = Mth<double, R>::exp(y1 * lx);
    r2 = Mth<double, R>::exp(y2 * lx);
    return;
  }
#endif
#endif
  r1 = Mth<T, R>::pow(x, y1);
  r2 = Mth<T, R>::pow(x, y2);
}

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

// NMP_SQRT_SHORT=0: the range-proven sqrt sites keep the IEEE lowering (A/B probe)
#ifndef NMP_SQRT_SHORT
#define NMP_SQRT_SHORT 1
#endif
// Division in the Newton loops (vege_flux, bare_flux, sfcdif1, ragrb).  fp32
// (the bit-exact path): IEEE `/`, except at the range-proven sites that go
// through DivFast32 (below).  fp64 (held to tolerances, not bits): the
// reciprocal from v_rcp_f64 refined by two Newton steps, times the numerator,
// plus one residual correction -- within 1 ulp of the IEEE quotient, in 9
// instructions instead of the div_scale/div_fmas/div_fixup sequence's 13, and
// without its vcc chain.  v_div_fixup_f64 gives zero, infinite and NaN
// operands (and overflow) their IEEE results and the quotient its sign.  (A
// branch back to IEEE `/` for non-finite results instead measured slower than
// plain `/`: profiles/r02/fp64_div.txt.)
// Valid range: the 1-ulp bound needs 1/b normal and the quotient and the
// residual b*q - a clear of underflow, i.e. 2^-1021 < |b| < 2^1021 and a
// normal quotient.  For |b| >= 2^1022 the reciprocal is subnormal or flushes
// and for subnormal b it overflows, so the result is NOT the IEEE quotient
// there (tests/test_gpu_routines.py pins both sides).  Every divisor these
// loops see is a physical resistance, conductance, temperature or height,
// many decades inside the range.
template <class T>
__device__ __forceinline__ T dv(T a, T b) {
  return a / b;
}
#if defined(NMP_F32_DIV) && NMP_F32_DIV == 1
// candidate: the IEEE lowering with ONE residual correction instead of two
template <>
__device__ __forceinline__ float dv<float>(float a, float b) {
  bool num_scaled;
  const float den = __builtin_amdgcn_div_scalef(a, b, false, &num_scaled);
  const float num = __builtin_amdgcn_div_scalef(a, b, true, &num_scaled);
  float r = __builtin_amdgcn_rcpf(den);
  const float e0 = __builtin_fmaf(-den, r, 1.0f);
  r = __builtin_fmaf(e0, r, r);
  const float q = num * r;
  const float e = __builtin_fmaf(-den, q, num);
  return __builtin_amdgcn_div_fixupf(__builtin_amdgcn_div_fmasf(e, r, q, num_scaled), b, a);
}
#elif defined(NMP_F32_DIV)
// timing probes of shorter fp32 division sequences (tools only, NOT shipped):
// 9 = v_rcp + one Newton step + two residual corrections + div_fixup (the IEEE
// sequence without div_scale / div_fmas), 7 = one residual correction
template <>
__device__ __forceinline__ float dv<float>(float a, float b) {
  float r = __builtin_amdgcn_rcpf(b);
  float e = __builtin_fmaf(-b, r, 1.0f);
  r = __builtin_fmaf(e, r, r);
  float q = a * r;
  e = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(e, r, q);
#if NMP_F32_DIV == 9
  e = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(e, r, q);
#endif
  return __builtin_amdgcn_div_fixupf(q, b, a);
}
#endif
template <>
__device__ __forceinline__ double dv<double>(double a, double b) {
#ifdef NMP_F64_IEEE_DIV
  return a / b;
#else
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  double q = a * r;
  e = __builtin_fma(-b, q, a);
  q = __builtin_fma(e, r, q);
#ifdef NMP_F64_DV_NOGUARD
  return q;
#else
  return __builtin_amdgcn_div_fixup(q, b, a);
#endif
#endif
}

// ---------------------------------------------------------------------------
// Division policies of the canopy Newton loop (vege_flux, with its sfcdif1 and
// ragrb).  Every a/b there goes through a policy object `d`:
//   Recip<T> R = d.rec(b);  the denominator and its reciprocal (shared by every
//                           division by the same value)
//   d.div(a, R)             a/b for any numerator
//   d.divk(a, R)            a/b for a numerator that is a constant or was passed
//                           through d.chk() (loop-invariant)
// DivRef is the reference's rounding: IEEE `/` in fp32 (the compiler's
// div_scale / div_fmas / div_fixup sequence, 11 instructions and a vcc chain
// per division), `dv` in fp64.
//
// DivFast32 below is the faster fp32 policy.  Round 3 guarded it dynamically
// (a per-division range check) and removed it: no faster than IEEE once
// guarded.  Round 4 proves its operands in range statically (tools/div_proof.py
// over the domain of vege_domain.h), checks that domain once per column plus a
// few windows per iteration, and re-runs the loop through DivRef for a lane
// outside it (DESIGN.md "Division in the Newton loops").
template <class T>
struct Recip {
  T b, r;
};

template <class T>
struct DivRef {
  __device__ __forceinline__ Recip<T> rec(T b) const { return {b, b}; }
  __device__ __forceinline__ T div(T a, const Recip<T>& R) const { return dv(a, R.b); }
  __device__ __forceinline__ T divk(T a, const Recip<T>& R) const { return dv(a, R.b); }
  __device__ __forceinline__ void chk(T) const {}
  // the reference's SQRT: IEEE correctly rounded
  __device__ __forceinline__ static T sqrt(T x) {
    if constexpr (sizeof(T) == 4) return ::sqrtf(x);
    else return ::sqrt(x);
  }
};

// sqrt of a finite x >= 2^-96: the compiler's
// correctly rounded fp32 sqrt sequence without its scaling of x < 2^-96 and
// its zero / infinity / NaN select, neither of which changes a result in that
// range.  v_sqrt_f32, then the two neighbour tests: s - 1 ulp if
// fma(-(s-ulp), s, x) <= 0, s + 1 ulp if fma(-(s+ulp), s, x) > 0 -- the same
// instructions in the same order as the IEEE lowering (tests/test_gpu_routines.py
// compares it with sqrtf over the range).
__device__ __forceinline__ float sqrt_normal32(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, s) - 1u);
  const float vm = __builtin_fmaf(-sm, s, x);
  float r = (vm <= 0.0f) ? sm : s;
  const float sp = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, s) + 1u);
  const float vp = __builtin_fmaf(-sp, s, x);
  return (vp > 0.0f) ? sp : r;
}

// DivFast32: the short exact sequence, used where the operands are proven to
// lie in its exact region (DESIGN.md "Division in the canopy loop").  The
// reciprocal r = fma(fma(-b, r0, 1), r0, r0) from v_rcp_f32 (shared by every
// division by the same b), then q = a*r, one fma residual correction and
// v_div_fixup_f32, which gives zero, infinite and NaN operands their IEEE
// results.  It equals IEEE a/b bit for bit whenever |b| is in [2^-126, 2^126]
// (normal, with a normal reciprocal), the residual a - b*q is not subnormal
// (a = 0 or |a| >= 2^-102) and |a/b| is in [2^-126, 2^126]
// (tools/fdiv_exhaust.hip: every normal b, every pair of significands, exact
// scaling by powers of two; profiles/r03/fdiv_exhaust2.txt; and the region's
// exponent edges, tests/test_gpu_routines.py).  The region stops short of
// FLT_MAX on purpose: for quotients within an ulp or two of it the product
// a*r can round past FLT_MAX and the sequence differs.
struct DivFast32 {
  __device__ __forceinline__ static float recip(float b) {
    float r = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, r, 1.0f);
    return __builtin_fmaf(e, r, r);
  }
#ifdef NMP_DIV_NOSHARE
  // (probe) no shared reciprocal: each quotient forms its own (fewer live
  // registers, three more instructions per division)
  __device__ __forceinline__ Recip<float> rec(float b) const { return {b, b}; }
  __device__ __forceinline__ float div(float a, const Recip<float>& R) const {
    const float r = recip(R.b);
    float q = a * r;
    const float e = __builtin_fmaf(-R.b, q, a);
    q = __builtin_fmaf(e, r, q);
    return __builtin_amdgcn_div_fixupf(q, R.b, a);
  }
#else
  __device__ __forceinline__ Recip<float> rec(float b) const { return {b, recip(b)}; }
  __device__ __forceinline__ float div(float a, const Recip<float>& R) const {
    float q = a * R.r;
    const float e = __builtin_fmaf(-R.b, q, a);
    q = __builtin_fmaf(e, R.r, q);
    return __builtin_amdgcn_div_fixupf(q, R.b, a);
  }
#endif
  __device__ __forceinline__ float divk(float a, const Recip<float>& R) const { return div(a, R); }
  __device__ __forceinline__ void chk(float) const {}
  // at the range-proven sqrt sites (tools/div_proof.py): x finite and >= 2^-96
  __device__ __forceinline__ static float sqrt(float x) {
#if NMP_SQRT_SHORT
    return sqrt_normal32(x);
#else
    return ::sqrtf(x);
#endif
  }
};

// Register-array access with a runtime index, lowered to a select chain so the
// array itself stays in VGPRs (a dynamic subscript would demote it to scratch).
// The empty asm pins each element as a register value: without it InstCombine
// folds the select chain back into one dynamically indexed load (a[i]), which
// forces the whole enclosing aggregate (the column struct) into scratch.
template <class T>
__device__ __forceinline__ T pin(T v) {
#ifdef NMP_PIN_NONVOLATILE
  __asm__("" : "+v"(v));
#else
  __asm__ volatile("" : "+v"(v));
#endif
  return v;
}
template <class T, int N>
__device__ __forceinline__ T dget(const T (&a)[N], int i) {
  T r = pin(a[0]);
#ifdef NMP_DGET_BRANCHY
  // (A/B only) the pin inside the select: the volatile asm cannot be
  // speculated, so every element becomes an exec-masked branch
#pragma unroll
  for (int k = 1; k < N; ++k) r = (i == k) ? pin(a[k]) : r;
#else
  // every element pinned unconditionally, then selected: one v_cndmask each
#pragma unroll
  for (int k = 1; k < N; ++k) {
    const T v = pin(a[k]);
    r = (i == k) ? v : r;
  }
#endif
  return r;
}
template <class T, int N>
__device__ __forceinline__ void dset(T (&a)[N], int i, T v) {
#pragma unroll
  for (int k = 0; k < N; ++k)
    if (i == k) a[k] = v;
}
// LDS-resident per-lane arrays (NMP_LDS_WORK): element k of lane t lives at
// pool[(SLOT + k) * NMP_BLOCK + t], i.e. [array][layer][lane] -- consecutive
// lanes hit consecutive banks, a runtime layer index is one address add, and
// the array holds no VGPRs across the step.  Each lane touches only its own
// column, so no barrier is needed.
template <class T>
__device__ __forceinline__ T* lds_lane_pool() {
  __shared__ T pool[NMP_LDS_SLOTS * NMP_BLOCK];
  return pool + threadIdx.x;
}
template <class T, int N, int SLOT>
struct LArr {
  static_assert(SLOT + N <= NMP_LDS_SLOTS, "LDS slot pool too small");
  __device__ __forceinline__ T& operator[](int k) const {
    return lds_lane_pool<T>()[(SLOT + k) * NMP_BLOCK];
  }
};
template <class T, int N, int S>
__device__ __forceinline__ T dget(const LArr<T, N, S>& a, int i) { return a[i]; }
template <class T, int N, int S>
__device__ __forceinline__ void dset(const LArr<T, N, S>& a, int i, T v) { a[i] = v; }

__device__ __forceinline__ float zget(const float (&a)[4], int i) {
  return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

}  // namespace nmp

// literal in the working precision: fp32 literals are parsed as float (like the
// reference's default-real constants), fp64 literals as double
#define L(x) (sizeof(T) == 4 ? (T)(x##f) : (T)(x))
