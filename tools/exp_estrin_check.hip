// fp64 exp_estrin (csrc/sflx_math.h) against the host exp over [-750, 710]
// and the special cases (GPU box; built by hand: hipcc -O3
// --offload-arch=gfx950 -I noahmp-1_amd/csrc -I include -o tools/exp_estrin_check
// tools/exp_estrin_check.hip).  Prints the maximum relative error in ulp.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include "sflx_kargs.h"
#include "sflx_math.h"
__global__ void k(int n, const double* x, double* a, double* b) {
  int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
  a[i] = nmp::exp_estrin(x[i]); b[i] = exp(x[i]);
}
int main() {
  const int n = 1 << 22; std::vector<double> x(n), a(n), b(n);
  for (int i = 0; i < n; ++i) x[i] = -750.0 + 1460.0 * (double)i / n;
  x[0] = 0; x[1] = NAN; x[2] = INFINITY; x[3] = -INFINITY; x[4] = 1e-300; x[5] = 709.7; x[6]=-745.0;
  double *dx, *da, *db; hipMalloc(&dx, n*8); hipMalloc(&da, n*8); hipMalloc(&db, n*8);
  hipMemcpy(dx, x.data(), n*8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n/256), dim3(256), 0, 0, n, dx, da, db);
  hipMemcpy(a.data(), da, n*8, hipMemcpyDeviceToHost); hipMemcpy(b.data(), db, n*8, hipMemcpyDeviceToHost);
  double maxrel = 0; long bad = 0;
  for (int i = 0; i < n; ++i) {
    double ref = std::exp(x[i]);
    if (std::isnan(ref)) { if (!std::isnan(a[i])) ++bad; continue; }
    if (ref == 0 || std::isinf(ref)) { if (a[i] != ref && std::fabs(ref) > 1e-300) ++bad; continue; }
    if (ref < 1e-300) continue;
    double rel = std::fabs(a[i] - ref) / ref; if (rel > maxrel) maxrel = rel;
  }
  printf("exp_estrin: max rel err vs host exp %.3g (%.2f ulp), special-case mismatches %ld\n", maxrel, maxrel / 2.22e-16, bad);
  return 0;
}
