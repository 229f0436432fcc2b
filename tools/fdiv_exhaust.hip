// Exhaustive check of the short fp32 division sequences against IEEE `/` on
// the GPU itself (the hardware v_rcp_f32 cannot be emulated on the host).
//
//   T1  every finite normal b (both signs, 2^32 patterns minus specials):
//       r1 = fma(fma(-b, r0, 1), r0, r0), r0 = v_rcp_f32(b), against the
//       correctly rounded 1.0f / b -- is one Newton step from v_rcp always
//       the correctly rounded reciprocal?
//   T2  every pair of significands a, b in [1, 2) (2^46 pairs): the 7-
//       instruction sequence (q0 = a*r1, one fma residual correction,
//       v_div_fixup) and the 9-instruction one (two corrections) against
//       IEEE a / b.  With T1 exact, every step is scale-invariant in the
//       normal range, so T2 covers all operands whose intermediates stay
//       normal (csrc/sflx_math.h states that range).
//   T3  random operands over the whole exponent range and special values,
//       split by whether they are inside that range.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/fdiv_exhaust tools/fdiv_exhaust.hip
//   tools/fdiv_exhaust [T2 launches to run, default 64 = all]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

__device__ __forceinline__ float rcp1(float b) {
  float r = __builtin_amdgcn_rcpf(b);
  float e = __builtin_fmaf(-b, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float div7(float a, float b) {
  const float r = rcp1(b);
  float q = a * r;
  const float e = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(e, r, q);
  return __builtin_amdgcn_div_fixupf(q, b, a);
}
__device__ __forceinline__ float div9(float a, float b) {
  const float r = rcp1(b);
  float q = a * r;
  float e = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(e, r, q);
  e = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(e, r, q);
  return __builtin_amdgcn_div_fixupf(q, b, a);
}
// the IEEE lowering (div_scale / div_fmas keep every operand in range) with
// ONE residual correction instead of two: 9 instructions instead of 11
__device__ __forceinline__ float div_cr9(float a, float b) {
  bool num_scaled;
  const float den = __builtin_amdgcn_div_scalef(a, b, false, &num_scaled);
  const float num = __builtin_amdgcn_div_scalef(a, b, true, &num_scaled);
  const float r = rcp1(den);
  const float q = num * r;
  const float e = __builtin_fmaf(-den, q, num);
  const float qs = __builtin_amdgcn_div_fmasf(e, r, q, num_scaled);
  return __builtin_amdgcn_div_fixupf(qs, b, a);
}
__device__ __forceinline__ bool same(float x, float y) {
  return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y);
}

// T1: one thread per 2^32/grid slice of bit patterns
__global__ void t1(unsigned long long* bad, unsigned* first) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long nbad = 0;
  for (uint64_t u = tid; u < (1ull << 32); u += nthr) {
    const float b = __uint_as_float((unsigned)u);
    const unsigned ex = ((unsigned)u >> 23) & 0xff;
    if (ex == 0 || ex == 0xff || ex >= 253) continue;  // normal b with normal 1/b
    const float r = rcp1(b);
    const float w = 1.0f / b;
    if (!same(r, w)) {
      ++nbad;
      atomicMin(first, (unsigned)u);
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

// T1b: rcp1 is exponent-independent: rcp1(m * 2^k) == rcp1(m) * 2^-k for every
// significand m in [1, 2) and every k with m*2^k and its reciprocal normal
__global__ void t1b(unsigned long long* bad) {
  const unsigned mb = blockIdx.x * blockDim.x + threadIdx.x;
  if (mb >= (1u << 23)) return;
  const float m = __uint_as_float(0x3f800000u | mb);
  const float r = rcp1(m);
  unsigned long long n = 0;
  for (int k = -125; k <= 125; ++k) {
    const float rk = rcp1(ldexpf(m, k));
    if (!same(rk, ldexpf(r, -k))) ++n;
  }
  if (n) atomicAdd(bad, n);
}

// T2: thread = one b significand, loops over a slice of a significands
__global__ void t2(unsigned a0, unsigned na, unsigned long long* bad7,
                   unsigned long long* bad9, unsigned* ex7) {
  const unsigned mb = blockIdx.x * blockDim.x + threadIdx.x;  // 0 .. 2^23-1
  if (mb >= (1u << 23)) return;
  const float b = __uint_as_float(0x3f800000u | mb);
  unsigned long long n7 = 0, n9 = 0;
  for (unsigned k = 0; k < na; ++k) {
    const float a = __uint_as_float(0x3f800000u | (a0 + k));
    const float w = a / b;
    if (!same(div7(a, b), w)) {
      ++n7;
      ex7[0] = a0 + k;
      ex7[1] = mb;
    }
    if (!same(div9(a, b), w)) ++n9;
    if (!same(div_cr9(a, b), w)) ++n9;
  }
  if (n7) atomicAdd(bad7, n7);
  if (n9) atomicAdd(bad9, n9);
}

// T3: random operand pairs; class 0 = inside the stated range, 1 = outside
__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
__device__ bool in_range(float a, float b) {
  const float fa = fabsf(a), fb = fabsf(b);
  if (!(fb >= 0x1p-60f && fb <= 0x1p60f)) return false;
  if (fa == 0.0f) return true;
  return fa >= 0x1p-60f && fa <= 0x1p60f;
}
__global__ void t3(uint64_t seed, int n_per, unsigned long long* cnt) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long c[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // [in,out] x {n, bad7, bad9}, cr9 bad
  for (int i = 0; i < n_per; ++i) {
    const uint64_t h = mix(seed ^ mix(tid * 7919 + i));
    float a = __uint_as_float((unsigned)h), b = __uint_as_float((unsigned)(h >> 32));
    if ((h & 0xf00) == 0) a = 0.0f * (h & 1 ? -1.0f : 1.0f);
    const int k = in_range(a, b) ? 0 : 3;
    const float w = a / b;
    ++c[k];
    if (!same(div7(a, b), w)) ++c[k + 1];
    if (!same(div9(a, b), w)) ++c[k + 2];
    if (!same(div_cr9(a, b), w)) ++c[6 + k / 3];
  }
  for (int k = 0; k < 8; ++k)
    if (c[k]) atomicAdd(&cnt[k], c[k]);
}

int main(int argc, char** argv) {
  const int t2_launches = argc > 1 ? std::atoi(argv[1]) : 64;
  unsigned long long* d;
  unsigned* u;
  CHECK(hipMalloc(&d, 16 * sizeof(unsigned long long)));
  CHECK(hipMalloc(&u, 4 * sizeof(unsigned)));
  CHECK(hipMemset(d, 0, 16 * sizeof(unsigned long long)));
  unsigned init[4] = {0xffffffffu, 0, 0, 0};
  CHECK(hipMemcpy(u, init, sizeof(init), hipMemcpyHostToDevice));

  hipLaunchKernelGGL(t1, dim3(65536), dim3(256), 0, 0, d, u);
  CHECK(hipDeviceSynchronize());
  unsigned long long h[16];
  unsigned hu[4];
  CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hu, u, sizeof(hu), hipMemcpyDeviceToHost));
  std::printf("T1 reciprocal (rcp + 1 Newton step) vs 1.0f/b over all normal b, |1/b| normal: "
              "%llu mismatches%s", h[0], h[0] ? "" : "\n");
  if (h[0]) std::printf(" (first 0x%08x)\n", hu[0]);
  std::fflush(stdout);

  hipLaunchKernelGGL(t1b, dim3((1u << 23) / 256), dim3(256), 0, 0, d + 3);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  std::printf("T1b rcp1(m 2^k) == rcp1(m) 2^-k for all m in [1,2), |k| <= 125: %llu mismatches\n",
              h[3]);
  std::fflush(stdout);

  // T2: a significands in t2_launches slices of 2^23/64
  const unsigned slice = (1u << 23) / 64;
  for (int L = 0; L < t2_launches && L < 64; ++L) {
    hipLaunchKernelGGL(t2, dim3((1u << 23) / 256), dim3(256), 0, 0, L * slice, slice, d + 1, d + 2,
                       u + 1);
    CHECK(hipDeviceSynchronize());
    if (L % 8 == 7 || L == t2_launches - 1) {
      CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
      std::printf("T2 %2d/64 slices: div7 mismatches %llu, div9 + cr9 mismatches %llu\n", L + 1,
                  h[1], h[2]);
      std::fflush(stdout);
    }
  }
  CHECK(hipMemcpy(hu, u, sizeof(hu), hipMemcpyDeviceToHost));
  if (h[1]) std::printf("   last div7 mismatch: a significand 0x%06x b significand 0x%06x\n", hu[1],
                        hu[2]);
  const double pairs = (double)std::min(t2_launches, 64) * slice * (double)(1u << 23);
  std::printf("T2 covered %.4g significand pairs (all: %.4g)\n", pairs, std::ldexp(1.0, 46));

  hipLaunchKernelGGL(t3, dim3(4096), dim3(256), 0, 0, 12345ull, 4096, d + 8);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  std::printf("T3 random pairs inside |a| in {0} U [2^-60,2^60], |b| in [2^-60,2^60]: %llu, "
              "div7 bad %llu, div9 bad %llu\n", h[8], h[9], h[10]);
  std::printf("T3 random pairs outside that range (incl. inf/nan/subnormal): %llu, div7 bad %llu, "
              "div9 bad %llu\n", h[11], h[12], h[13]);
  std::printf("T3 cr9 (div_scale + one correction + div_fmas) bad: inside %llu, outside %llu\n",
              h[14], h[15]);
  return 0;
}
