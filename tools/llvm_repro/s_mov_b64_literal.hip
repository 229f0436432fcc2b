// Reduced reproducer: with -mllvm -disable-machine-cse the
// AMDGPU backend of ROCm 7.2's LLVM emits, for gfx950,
//     s_mov_b64 s[0:1], 0x4049000000000000      ; 50.0 as a double
// an SALU 64-bit move of a 64-bit immediate that gfx950 cannot encode: the
// text assembler rejects it ("invalid operand for instruction"), and the
// integrated assembler silently encodes the literal's LOW 32 bits (here 0),
// so s[0:1] = 0.0 and `c * 50.0` becomes 0.  Instruction selection produces
// S_MOV_B64 with the 64-bit immediate in MIR (llc -print-after=amdgpu-isel);
// normally SI Fold Operands folds it into its f64 VALU users (where a 32-bit
// literal holds the high half) and it disappears; without MachineCSE a copy
// of the constant survives into an SGPR pair that a VALU instruction reads.
//
// In the engine the same thing hit ocml's double exp (its 1024.0 overflow
// bound became 0, so exp(x) = inf for every x > 0) and sqrt's scaling bound
// in the spilling fp64 step kernels: ragrb's exp(CWPC) (func.f90 ragrb) went
// to inf, hence RAHG = inf and NaN states (profiles/r03/mcse_*.txt).
//
// Build and run: tools/llvm_repro/run.sh (CPU part anywhere; the GPU part
// on an MI355X).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void k(const double* x, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double c = sqrt(x[i]);
  out[i] = c * 50.0 + 1.0;
}

int main() {
  const int n = 256;
  double hx[n], ho[n];
  for (int i = 0; i < n; ++i) hx[i] = 1.0 + i;
  double *dx, *dout;
  if (hipMalloc(&dx, sizeof(hx)) != hipSuccess || hipMalloc(&dout, sizeof(ho)) != hipSuccess)
    return 2;
  hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(n), 0, 0, dx, dout, n);
  hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i)
    if (std::fabs(ho[i] - (std::sqrt(hx[i]) * 50.0 + 1.0)) > 1e-9) ++bad;
  std::printf("out[3] = %.6f (expected %.6f); %d of %d wrong\n", ho[3], std::sqrt(hx[3]) * 50.0 + 1.0,
              bad, n);
  return bad ? 1 : 0;
}
