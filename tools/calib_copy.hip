// PMC calibration for the engine's access pattern: SoA field-major fp32,
// one lane per column, 4 B per lane per field (exactly how sflx_step_kernel
// reads/writes state).  Reads NF fields of N columns and writes them back
// (+1), so the algorithmic traffic is NF*N*4 B read + NF*N*4 B written.
// Run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE; tools/pmc_traffic.py
// turns the counter/byte ratio into the correction applied to the engine.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int NF = 56;

__global__ __launch_bounds__(256) void calib_soa_copy(float* __restrict__ a, long n) {
  long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  float v[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) v[f] = a[(long)f * n + c];
#pragma unroll
  for (int f = 0; f < NF; ++f) a[(long)f * n + c] = v[f] + 1.0f;
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : (1L << 20);
  int reps = argc > 2 ? atoi(argv[2]) : 5;
  float* a;
  if (hipMalloc(&a, sizeof(float) * NF * n) != hipSuccess) return 2;
  (void)hipMemset(a, 0, sizeof(float) * NF * n);
  for (int r = 0; r < reps; ++r)
    calib_soa_copy<<<(n + 255) / 256, 256>>>(a, n);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  printf("calib_soa_copy n=%ld fields=%d bytes_read=%ld bytes_written=%ld per launch\n", n, NF,
         (long)NF * n * 4, (long)NF * n * 4);
  (void)hipFree(a);
  return 0;
}
