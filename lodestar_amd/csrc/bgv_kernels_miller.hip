// k_miller in its own translation unit, a tuning variant:
//   python -m lodestar_amd.build --variant NAME BGV_MILLER_SPLIT [BGV_MILLER_MUL_CALLS]
// miller_loop2 is inlined into the kernel, and fp_mul/fp_sqr too unless
// -DBGV_MILLER_MUL_CALLS.  This unit compiles in ~1 min (with calls) or ~5 min (inlined)
// against ~5 min for bgv_kernels.hip, so Miller-loop experiments are cheap.  The header
// functions that stay out of line are static here, so the host objects do not collide
// with bgv_kernels.hip's.  Measured: inlined products 41.0 -> 54.7 ms
// per 131,072 slots (more spills), calls kept: unchanged; the default build keeps
// k_miller in bgv_kernels.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BGV_NOINLINE static __host__ __device__ __noinline__
#ifndef BGV_MILLER_MUL_CALLS
#define BGV_MUL_ATTR __host__ __device__ __forceinline__
#endif
#define BGV_MILLER_LOOP_ATTR __host__ __device__ __forceinline__

#include "bgv_layout.h"
#define BGV_KERNEL_SIDE 1
#include "bls_pairing.h"

#ifndef BGV_WPE
#define BGV_WPE 1
#endif
#define BGV_KATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE, BGV_WPE)))

extern "C" {
#include "bgv_miller_kernel.h"
}
