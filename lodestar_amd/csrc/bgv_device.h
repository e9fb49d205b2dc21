// Device-side pieces shared by the kernel translation units (bgv_k_*.hip): the record
// layouts, the arithmetic headers, launch attributes, wavefront exchange helpers and
// the slot predicate.  Each kernel unit is compiled on its own (no device linking), so
// every unit carries its own copy of the out-of-line arithmetic with its own register
// budget: the per-set units are not constrained by each other's occupancy targets.
#pragma once
#include <stdlib.h>
#include "bgv_layout.h"
#define BGV_KERNEL_SIDE 1
#include "bls_hash.h"
#include "bls_pairing.h"
#include "bls_team.h"

// Waves per SIMD the verify kernels are register-budgeted for (1: up to 512 VGPRs).
#ifndef BGV_WPE
#define BGV_WPE 1
#endif
// k_prep: one wave per SIMD since the lazy point formulas (bls_lazy.h): 15.0 vs 16.1 ms per
// 64,512-set call (profiles/r02s3/roof_p1_*.json); two waves per SIMD were faster (36.6 vs
// 45.3 ms per 131,072 slots) with the eager formulas.  k_miller at two waves: 22.3 vs 11.7 ms.
#ifndef BGV_WPE_PREP
#define BGV_WPE_PREP 1
#endif
// Sets with at least this many cached pubkeys are aggregated by a tree (k_pk_agg16 on a
// 16-lane team up to BGV_PK_TEAM_MAX keys, k_pk_agg on a whole wave above) instead of
// serially on the set's k_prep lane.
#ifndef BGV_PK_TREE_MIN
#define BGV_PK_TREE_MIN 16
#endif
#ifndef BGV_PK_TEAM_MAX
#define BGV_PK_TEAM_MAX 256
#endif
#define BGV_KATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE, BGV_WPE)))
#define BGV_KATTR_PREP __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE_PREP, BGV_WPE_PREP)))

// Wavefront exchange of one 32-bit word with lane (l ^ m): ds_swizzle in bit-mask mode
// within each 32-lane half (m < 32), ds_bpermute across the halves (m = 32).  No LDS
// storage is allocated: both go through the LDS crossbar only.
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
  if constexpr (M == 32)
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((threadIdx.x ^ 32u) << 2), (int)v);
  else
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1f | (M << 10));  // and 0x1f, xor M
}

template <int M, class P>
__device__ __forceinline__ P point_xor(const P& p) {
  constexpr int W = (int)(sizeof(P) / 4);
  P r;
  const uint32_t* a = reinterpret_cast<const uint32_t*>(&p);
  uint32_t* o = reinterpret_cast<uint32_t*>(&r);
  BGV_UNROLL for (int i = 0; i < W; ++i) o[i] = lane_xor<M>(a[i]);
  return r;
}



// slot first_slot + k is in group g (the mask covers the first 64; a longer run -- the
// partials of bgv_final_verify -- has every element in)
__device__ __forceinline__ bool grp_has(const bgv_dgroup& g, uint32_t k) {
  return k < g.n_slots && (k >= 64 || ((g.mask >> k) & 1));
}

// A slot takes part in its group's equation iff it is a set whose signature decoded
// (valid or infinity) and whose pubkeys aggregated to a finite point; its signature
// joins the group's sum only when it is not the infinity signature (blst skips those).
__device__ __forceinline__ bool slot_live(const bgv_dslot& d, int32_t ss, int32_t ps) {
  return !(d.flags & BGV_SLOT_PAD) && (ss == BGV_ST_OK || ss == BGV_ST_INFINITY) && ps == BGV_ST_OK;
}

#include "bgv_launch.h"

static inline unsigned nblk(uint32_t n, unsigned t) { return (n + t - 1) / t; }

// sets up to which the latency path's team work runs one set per block and task (k_prep_wide,
// 4 blocks per set) instead of four sets per block (k_prep_team), and the first pass pairs
// each signature on its own (bgv_sig_pairs): a couple of rounds of waves on the chip
#define BGV_PREP_WIDE_MAX 340
// pairs up to which the latency path runs one Miller loop per block (k_miller_wide) instead of
// four (k_miller_team)
#define BGV_MILLER_WIDE_MAX 1024

// Latency path (small calls): at most this many pairs (sets + groups) take the split
// k_prep_a / k_prep_team and the team Miller loop instead of one lane per set and task, which
// wins while the chip would otherwise sit mostly idle (one lane per set runs ~13 ms in
// k_miller however small the call).  BGV_LATENCY_MAX overrides (0 disables).
static inline uint32_t bgv_latency_max() {
  static const uint32_t v = [] {
    const char* e = getenv("BGV_LATENCY_MAX");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 16384u;
  }();
  return v;
}

// the latency path's kernels for this batch: forced by b.path, else by size
static inline bool bgv_use_latency(const bgv_dev_batch& b, uint32_t pairs) {
  return b.path == BGV_PATH_LATENCY || (b.path == BGV_PATH_AUTO && pairs <= bgv_latency_max());
}

// Kernel k of a verify launch is bracketed by events kev[2k], kev[2k+1] when profiling.
#define BGV_MARK(i) \
  if (s.kev) (void)hipEventRecord(s.kev[i], s.main)
