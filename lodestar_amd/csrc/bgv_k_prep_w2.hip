// The bulk k_prep's sig and pk tasks compiled for two waves per SIMD (256 registers each), in
// a unit of their own so the budget applies to every function they call (bgv_k_prep_bulk.hip
// keeps one wave per SIMD).  Launched per task when BGV_PREP_W2 names it (bgv_launch_prep_bulk).
#include "bgv_k_tasks.h"

#define BGV_KATTR_W2 __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))

extern "C" {

__global__ void BGV_KATTR_W2 k_prep_sig2(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                         g2_jac* __restrict__ rsig, int32_t* __restrict__ sig_status) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < nslots) task_sig(s, slots, rsig, sig_status);
}

__global__ void BGV_KATTR_W2 k_prep_pk2(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                        const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                        const uint8_t* __restrict__ pk_bytes, g1_jac* __restrict__ rpk,
                                        int32_t* __restrict__ pk_status, const g1_jac* __restrict__ pk_agg) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < nslots) task_pk(s, slots, pk_idx, cache, pk_bytes, rpk, pk_status, pk_agg);
}

}  // extern "C"

hipError_t bgv_launch_prep_w2(const bgv_dev_batch& b, const bgv_streams& s, bool tree, int task) {
  if (task == 1)
    hipLaunchKernelGGL(k_prep_sig2, dim3(nblk(b.nslots, 64)), dim3(64), 0, s.main, b.slots, b.nslots, b.rsig,
                       b.sig_status);
  else
    hipLaunchKernelGGL(k_prep_pk2, dim3(nblk(b.nslots, 64)), dim3(64), 0, s.main, b.slots, b.nslots, b.pk_idx,
                       reinterpret_cast<const g1_aff*>(b.cache_opaque), b.pk_bytes, b.rpk, b.pk_status,
                       tree ? b.pk_agg : nullptr);
  return hipGetLastError();
}
