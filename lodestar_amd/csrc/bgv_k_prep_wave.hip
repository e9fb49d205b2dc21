// The latency path's first per-set kernel for the smallest calls (up to BGV_PREP_WIDE_MAX sets,
// bgv_launch_prep): one set per 64-lane block and task, every lane holding the same values, so
// every Fp product runs on the whole wave -- BGV_WAVE_UNIFORM_MUL makes fp_mul / fp_sqr
// bgv_wfp.h's wfp_umul (one limb per lane, ~200 VALU instructions on the wave's chain instead
// of ~490 on one lane) and the square roots' exponentiations stay in the limb-per-lane form
// (bgv_pow_wave).  Planes (blockIdx.y): 0 / 1 the SSWU map + isogeny of u0 / u1, 2 the
// signature's decoding; the same tasks and formulas as k_prep_a's lane planes (bgv_k_lat.h).
#ifndef BGV_PREP_WAVE_LANE_MUL  // A/B: the other products on one lane's schedule (bgv_pow_wave only)
#define BGV_WAVE_UNIFORM_MUL 1
#endif
#include "bgv_k_lat.h"
#include "bgv_wfp.h"

extern "C" __global__ void __launch_bounds__(64) k_prep_a_wave(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                                               g2_jac* __restrict__ h, fp12_t* __restrict__ f,
                                                               int32_t* __restrict__ sig_status) {
  const uint32_t s = blockIdx.x;  // grid.x = nslots
  const bool w = threadIdx.x == 0;
  if (blockIdx.y == 0)
    task_map_t<bgv_pow_wave>(s, 0, slots, h + s, w);
  else if (blockIdx.y == 1)
    task_map_t<bgv_pow_wave>(s, 1, slots, split_q1(f, s), w);
  else
    task_sig_decode_t<bgv_pow_wave>(s, slots, split_sig(f, s), sig_status, w);
}

hipError_t bgv_launch_prep_wave(const bgv_dev_batch& b, hipStream_t st) {
  if (b.nslots == 0) return hipSuccess;
  hipLaunchKernelGGL(k_prep_a_wave, dim3(b.nslots, 3), dim3(64), 0, st, b.slots, b.nslots, b.h, b.f, b.sig_status);
  return hipGetLastError();
}
