// The fp64 half-occupancy ("small") kernels' translation unit: sflx_kernel.hip
// compiled for NMP_TU 9 with MachineLICM on (build.py SOURCE_FLAGS), while
// the fp64 full-occupancy kernels (NMP_TU 8) and the fp32 ones (NMP_TU 4)
// keep it off.  Config #2 (65,536 fp64 columns, one wave per SIMD) runs this
// kernel.
#define NMP_TU 9
#include "sflx_kernel.hip"
