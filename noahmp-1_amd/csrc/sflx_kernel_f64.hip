// The fp64 kernels' translation unit: sflx_kernel.hip compiled for NMP_TU 8,
// in parallel with the fp32 unit (sflx_kernel.hip itself, NMP_TU 4), and
// with flags of its own where a tuning variant asks for them (build.py
// SOURCE_FLAGS, tools/build_variants.py f64*).  The fp32 kernels are the
// bit-exact path; the fp64 ones are held to tolerances (DESIGN.md "fp64").
#define NMP_TU 8
#include "sflx_kernel.hip"
