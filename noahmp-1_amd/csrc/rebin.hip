// Column re-binning: a per-tile counting sort of the columns
// by the loop-cost key the step kernel recorded (the vege_flux Newton trip
// count, func.f90:2744-2877 with its exit rule :2870-2875).
//
// The wave runs its slowest lane, so a wave whose 64 columns need 3..20
// Newton iterations runs 20.  Sorting each tile of `tile` consecutive columns
// by the previous step's trip count puts columns of similar cost into the
// same waves; the next step's launch reads the permutation (KArgs::order) and
// steps column order[i] on lane i.  The sort is tile-local so that the
// permuted loads and stores of a workgroup stay inside one tile's span of each
// field (a few KiB), and the permutation never leaves the tile.
//
// One 256-thread workgroup per tile: histogram of the keys in LDS, exclusive
// scan, then each column takes the next slot of its key's bucket.  Slots
// within a bucket are handed out by LDS atomics, so the order inside a bucket
// varies from run to run; no result depends on it.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace nmp {

constexpr int kRebinBuckets = 32;  // keys >= 31 share the last bucket

__global__ __launch_bounds__(256) void rebin_order_kernel(const uint8_t* __restrict__ cost,
                                                          int32_t* __restrict__ order,
                                                          int64_t ncol, int tile) {
  __shared__ int slot[kRebinBuckets];
  const int64_t base = (int64_t)blockIdx.x * tile;
  const int n = (int)((ncol - base) < tile ? (ncol - base) : tile);
  if (threadIdx.x < kRebinBuckets) slot[threadIdx.x] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int k = cost[base + i] < kRebinBuckets ? cost[base + i] : kRebinBuckets - 1;
    atomicAdd(&slot[k], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int k = 0; k < kRebinBuckets; ++k) {
      const int c = slot[k];
      slot[k] = s;
      s += c;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int k = cost[base + i] < kRebinBuckets ? cost[base + i] : kRebinBuckets - 1;
    const int p = atomicAdd(&slot[k], 1);
    order[base + p] = (int32_t)(base + i);
  }
}

hipError_t launch_rebin(const uint8_t* cost, int32_t* order, int64_t ncol, int tile,
                        hipStream_t stream) {
  const int64_t grid = (ncol + tile - 1) / tile;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(rebin_order_kernel, dim3((unsigned)grid), dim3(256), 0, stream, cost, order,
                     ncol, tile);
  return hipGetLastError();
}

}  // namespace nmp
