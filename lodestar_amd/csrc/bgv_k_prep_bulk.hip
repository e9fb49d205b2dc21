// The bulk preparation kernel of a verify call (gfx950), in a unit of its own so that its
// register budget (BGV_WPE_PREP waves per SIMD) applies to every function it calls: a
// device function shared with a kernel of another budget is compiled for the larger one.
//
//   k_prep  three independent tasks side by side (blockIdx.y): hash (H(m_i)), sig (decode,
//           subgroup check, r_i * sig_i) and pk (aggregate, r_i * pk_i); see bgv_k_tasks.h
// Fp2 products with deferred reduction (bls_wide.h); every kernel of this unit runs 64-thread
// blocks, as the products' per-lane LDS operand slot requires
#ifndef BGV_LZ2_CLASSIC
#define BGV_LZ2_WIDE 1
#define BGV_LZ2_WIDE_STRICT 1  // no silent fallback to the fully reduced product
#endif
#include "bgv_k_tasks.h"

// waves per SIMD the bulk k_prep is register-budgeted for (1: 512 registers, 2: 256)
#ifndef BGV_WPE_BULK
#define BGV_WPE_BULK 1
#endif
#define BGV_KATTR_BULK __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE_BULK, BGV_WPE_BULK)))

extern "C" {

// The three independent per-set tasks in one launch (blockIdx.y = task), so one
// batch keeps 3x the wavefronts in flight on a single stream.
__global__ void BGV_KATTR_BULK k_prep(const bgv_dslot* __restrict__ slots, uint32_t nslots, g2_jac* __restrict__ rsig,
                                      int32_t* __restrict__ sig_status, g2_jac* __restrict__ h,
                                      const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                      const uint8_t* __restrict__ pk_bytes, g1_jac* __restrict__ rpk,
                                      int32_t* __restrict__ pk_status, const g1_jac* __restrict__ pk_agg,
                                      const uint32_t* __restrict__ uniq, uint32_t nuniq, uint32_t task0) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t task = blockIdx.y + task0;
  // hash first: the longest task starts earliest.  With uniq, lane u hashes the u-th distinct
  // signing root (slot uniq[u]); lanes past nuniq -- whole waves of them -- exit at once.
  if (task == 0) {
    if (uniq) {
      if (s < nuniq) task_hash(uniq[s], slots, h);
    } else if (s < nslots) {
      task_hash(s, slots, h);
    }
    return;
  }
  if (s >= nslots) return;
  if (task == 1)
    task_sig(s, slots, rsig, sig_status);
  else
    task_pk(s, slots, pk_idx, cache, pk_bytes, rpk, pk_status, pk_agg);
}

}  // extern "C"

// BGV_PREP_SPLIT=1 (profiling only: per-task kernel time and counters): the three tasks as
// three launches of k_prep, one plane each, in the same order
hipError_t bgv_launch_prep_bulk(const bgv_dev_batch& b, const bgv_streams& s, bool tree) {
  static const bool split = [] {
    const char* e = getenv("BGV_PREP_SPLIT");
    return e && atoi(e) > 0;
  }();
  for (uint32_t t0 = 0; t0 < 3; t0 += split ? 1 : 3) {
    hipLaunchKernelGGL(k_prep, dim3(nblk(b.nslots, 64), split ? 1 : 3), dim3(64), 0, s.main, b.slots, b.nslots, b.rsig,
                       b.sig_status, b.h, b.pk_idx, reinterpret_cast<const g1_aff*>(b.cache_opaque), b.pk_bytes, b.rpk,
                       b.pk_status, tree ? b.pk_agg : nullptr, b.uniq, b.nuniq, t0);
  }
  return hipGetLastError();
}
