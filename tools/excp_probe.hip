// Does gfx950 record floating-point exception status (TRAPSTS.EXCP, sticky)
// with the traps disabled?  If so, one s_getreg after a stretch of fast
// arithmetic tells a wave whether any lane under- or overflowed, a wave-level
// guard for division sequences that are exact only in the normal range.
//   hipcc -O3 --offload-arch=gfx950 -o tools/excp_probe tools/excp_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

// hwreg(HW_REG_TRAPSTS = 3, offset 0, size 9): EXCP[8:0]
#define TRAPSTS_EXCP (3 | (0 << 6) | ((9 - 1) << 11))
// MODE (id 1) whole register
#define MODE_ALL (1 | (0 << 6) | ((32 - 1) << 11))

__global__ void probe(const float* in, int op, unsigned* out) {
  const int t = threadIdx.x;
  __builtin_amdgcn_s_setreg(TRAPSTS_EXCP, 0);
  const unsigned before = __builtin_amdgcn_s_getreg(TRAPSTS_EXCP);
  float a = in[t], b = in[64 + t];
  float x;
  if (op == 0) x = a * b;                         // per-lane inputs decide the exception
  else if (op == 1) x = __builtin_amdgcn_rcpf(b);
  else if (op == 2) x = __builtin_fmaf(a, b, -a);
  else x = a + b;
  out[128 + t] = __float_as_uint(x);
  __builtin_amdgcn_s_waitcnt(0);
  __asm__ volatile("s_nop 7\n s_nop 7" ::: "memory");
  const unsigned after = __builtin_amdgcn_s_getreg(TRAPSTS_EXCP);
  if (t == 0) {
    out[0] = before;
    out[1] = after;
    out[2] = __builtin_amdgcn_s_getreg(MODE_ALL);
  }
}

int main() {
  float h[128];
  unsigned* d_out;
  float* d_in;
  hipMalloc(&d_out, 256 * sizeof(unsigned));
  hipMalloc(&d_in, sizeof(h));
  struct Case { const char* name; int op; float a, b; int lane; };
  const Case cases[] = {
      {"clean 1.5*2", 0, 1.5f, 2.0f, -1},
      {"underflow 1e-30*1e-30 in lane 7", 0, 1.0f, 2.0f, 7},
      {"overflow 1e30*1e30 in lane 63", 0, 1.0f, 2.0f, 63},
      {"inexact 1/3*3", 0, 0.33333334f, 3.0f, -1},
      {"denormal input 1e-40*1", 0, 1.0f, 1.0f, 5},
      {"rcp(3e38) subnormal result", 1, 1.0f, 2.0f, 9},
      {"rcp(1e-40) denormal input", 1, 1.0f, 2.0f, 11},
      {"clean add", 3, 1.0f, 2.0f, -1},
  };
  for (int ci = 0; ci < 8; ++ci) {
    const Case& c = cases[ci];
    for (int i = 0; i < 64; ++i) {
      h[i] = c.a;
      h[64 + i] = c.b;
    }
    if (c.lane >= 0) {
      if (ci == 1) h[c.lane] = 1e-30f, h[64 + c.lane] = 1e-30f;
      if (ci == 2) h[c.lane] = 1e30f, h[64 + c.lane] = 1e30f;
      if (ci == 4) h[c.lane] = 1e-40f;
      if (ci == 5) h[64 + c.lane] = 3e38f;
      if (ci == 6) h[64 + c.lane] = 1e-40f;
    }
    hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
    hipMemset(d_out, 0xff, 256 * sizeof(unsigned));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_in, c.op, d_out);
    unsigned o[3];
    if (hipMemcpy(o, d_out, sizeof(o), hipMemcpyDeviceToHost) != hipSuccess) {
      std::printf("launch failed\n");
      return 1;
    }
    std::printf("%-32s EXCP before 0x%03x after 0x%03x   MODE 0x%08x\n", c.name, o[0], o[1], o[2]);
  }
  std::printf("EXCP bits: 0 invalid, 1 input denormal, 2 div by zero, 3 overflow, 4 underflow, "
              "5 inexact\n");
  return 0;
}
