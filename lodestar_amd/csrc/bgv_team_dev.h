// Device side of a team (bls_team.h): the LDS exchange of the coefficient-parallel Fp12
// operations, shared by the group closing (bgv_k_final.hip) and the team Miller loop
// (bgv_k_miller.hip).  One team = 16 lanes of a 64-lane block, BGV_FINAL_TEAMS per block
// (k_final12: 12 lanes, five teams per block).
#pragma once
#include "bgv_device.h"

#define BGV_FINAL_TEAMS (64 / BGV_TEAM)

// Group closing, team-parallel (bls_team.h): a team of 16 lanes per group, lane c < 12
// owning one Fp coefficient of the running value; operands exchanged through LDS.
static __constant__ fp2_t kTeamFrob1[6] = BGV_FROB1;
static __constant__ fp_t kTeamFrob2[6] = BGV_FROB2;

// T = lanes per team: 16 (lanes 12..15 duplicate 8..11; the team Miller loop's rounds use
// all 16) or 12 (k_final: five teams per wave)
template <int T>
struct tm_dev_ops_t {
  fp_t* A;  // this team's 12 + 12 LDS slots
  fp_t* B;
  int c;   // lane within the team, 0..T-1
  int cc;  // component computed by this lane
  __device__ fp_t mul(const fp_t& x, const fp_t& y) {
    if (c < BGV_TEAM_COMPS) {
      A[c] = x;
      B[c] = y;
    }
    __syncthreads();
    const fp_t r = tm_mul_lane(cc, A, B);
    __syncthreads();
    return r;
  }
  __device__ fp_t sqr(const fp_t& x) {
    if (c < BGV_TEAM_COMPS) A[c] = x;
    __syncthreads();
    const fp_t r = tm_sqr_lane(cc, A);
    __syncthreads();
    return r;
  }
  __device__ fp_t line(const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) { return tm_line_lane(cc, l0, l1, l3); }
  __device__ fp_t mul_line(const fp_t& x, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
    if (c < BGV_TEAM_COMPS) A[c] = x;
    __syncthreads();
    const fp_t r = tm_mul_line_lane(cc, A, l0, l1, l3);
    __syncthreads();
    return r;
  }
  __device__ fp_t conj(const fp_t& x) { return fp_select(((cc >> 1) & 1) != 0, x, fp_neg(x)); }
  __device__ fp_t frob(const fp_t& x) {
    if (c < BGV_TEAM_COMPS) A[c] = x;
    __syncthreads();
    const fp_t x0 = A[cc & ~1], x1 = A[cc | 1];
    __syncthreads();
    return tm_frob_lane(cc, x0, x1, kTeamFrob1[tm_tower_pos(cc)]);
  }
  __device__ fp_t frob2(const fp_t& x) { return fp_mul(x, kTeamFrob2[tm_tower_pos(cc)]); }
  __device__ bool is_fp6(const fp_t& x) {
    const bool bad = c < BGV_TEAM_COMPS && ((cc >> 1) & 1) && !fp_is_zero(x);
    const uint64_t m = __ballot(bad);
    return ((m >> ((threadIdx.x / T) * T)) & ((1ull << T) - 1)) == 0;
  }
};
using tm_dev_ops = tm_dev_ops_t<BGV_TEAM>;

// Synchronization of one wavefront's LDS exchange when the block holds other waves that run
// their own work (k_miller_wide): the fences of __syncthreads (the LDS stores complete, no
// compiler reordering across it) without the block barrier.  LDS operations of one wave are
// performed in order, so the wave's later reads see its earlier stores.  In a single-wave
// block this is what __syncthreads compiles to.
__device__ __forceinline__ void bgv_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// One Fp12 value per 64-lane block with the wide products (bls_team.h tm_mul_part): lane l
// holds coefficient c = l % 12 (replicated over q = l / 12); lanes q < 4 (l < 48) each compute
// a quarter of the double-width products of their coefficient, lanes 48..63 only keep the
// barriers.  A: 12 operand slots, B: 12, P: NP x 12 part slots (LDS).  WAVE: the value lives in
// one wave of a larger block, which synchronizes on its own (bgv_wave_sync).  NP = 8: the
// eight-part products (bls_team.h tm_mul_part8 ...), one double-width product per lane for a
// squaring or a line product, on a block of >= 96 lanes (k_final_fold).
template <bool WAVE, int NP = 4>
struct tm_wide_ops_t {
  fp_t* A;
  fp_t* B;
  fp_t* P;
  int c, q;
  __device__ void sync() {
    if (WAVE)
      bgv_wave_sync();
    else
      __syncthreads();
  }
  // Only the q == 0 lanes' values are ever read (every op takes its operands from them, and
  // the callers store and test their results), so in a block engine the others skip the part
  // sum: a wave without q == 0 lanes passes it by, the LDS reads shrink to the twelve lanes
  // that use them.  (A one-wave engine keeps the uniform form: k_miller_wide measured slower
  // with the branch, 0.60 vs 0.55 ms.)
  __device__ fp_t gather() {
    fp_t r = fp_zero();
    if (WAVE || q == 0) {
      if (NP == 8) {
        fp_t x[8];
        BGV_UNROLL for (int k = 0; k < 8; ++k) x[k] = P[k * BGV_TEAM_COMPS + c];
        r = tm_sum8(x);
      } else {
        r = tm_sum4(P[c], P[BGV_TEAM_COMPS + c], P[2 * BGV_TEAM_COMPS + c], P[3 * BGV_TEAM_COMPS + c]);
      }
    }
    return r;
  }
  __device__ fp_t mul(const fp_t& x, const fp_t& y) {
    if (q == 0) {
      A[c] = x;
      B[c] = y;
    }
    sync();
    if (q < NP) P[q * BGV_TEAM_COMPS + c] = NP == 8 ? tm_mul_part8(c, q, A, B) : tm_mul_part(c, q, A, B);
    sync();
    return gather();
  }
  __device__ fp_t sqr(const fp_t& x) {
    if (q == 0) A[c] = x;
    sync();
    if (q < NP) P[q * BGV_TEAM_COMPS + c] = NP == 8 ? tm_sqr_part8(c, q, A) : tm_sqr_part(c, q, A);
    sync();
    return gather();
  }
  __device__ fp_t mul_line(const fp_t& x, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
    if (q == 0) A[c] = x;
    sync();
    if (q < NP)
      P[q * BGV_TEAM_COMPS + c] =
          NP == 8 ? tm_mul_line_part8(c, q, A, l0, l1, l3) : tm_mul_line_part(c, q, A, l0, l1, l3);
    sync();
    return gather();
  }
  __device__ fp_t line(const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) { return tm_line_lane(c, l0, l1, l3); }
  __device__ fp_t conj(const fp_t& x) { return fp_select(((c >> 1) & 1) != 0, x, fp_neg(x)); }
  __device__ fp_t frob(const fp_t& x) {
    if (q == 0) A[c] = x;
    sync();
    const fp_t x0 = A[c & ~1], x1 = A[c | 1];
    sync();
    return tm_frob_lane(c, x0, x1, kTeamFrob1[tm_tower_pos(c)]);
  }
  __device__ fp_t frob2(const fp_t& x) { return fp_mul(x, kTeamFrob2[tm_tower_pos(c)]); }
  // The q == 0 lanes hold the value; the flag is reduced over the whole engine (the wave, or
  // the block with a block barrier), so every lane -- also those of a second wave, which hold
  // no q == 0 lane -- returns the same answer.  Every lane of the engine must call it.
  __device__ bool is_fp6(const fp_t& x) {
    const bool bad = q == 0 && ((c >> 1) & 1) && !fp_is_zero(x);
    if (WAVE) return __ballot(bad) == 0;
    return __syncthreads_or(bad ? 1 : 0) == 0;
  }
};
using tm_wide_ops = tm_wide_ops_t<false>;

// Eight-part ops with the lean squaring (bls_team.h tm_sqr_rec8): the lane's two operand
// recipes are fixed once, a squaring evaluates only them.  Same parts, bit for bit.
struct tm_wide8_lean_ops : tm_wide_ops_t<false, 8> {
  tm_lin_t rx, ry;
  __device__ fp_t sqr(const fp_t& x) {
    if (q == 0) A[c] = x;
    sync();
    if (q < 8) P[q * BGV_TEAM_COMPS + c] = tm_sqr_part8_lean(A, rx, ry);
    sync();
    return gather();
  }
};

// Four-part one-wave ops (k_miller_wide) with the lean squaring (bls_team.h tm_sqr_rec4):
// the lane's four operand recipes fixed once.  Same parts, bit for bit.
struct tm_wide4_lean_ops : tm_wide_ops_t<true, 4> {
  tm_lin_t x1, y1, x2, y2;
  __device__ fp_t sqr(const fp_t& x) {
    if (q == 0) A[c] = x;
    sync();
    if (q < 4) P[q * BGV_TEAM_COMPS + c] = tm_sqr_part4_lean(A, x1, y1, x2, y2);
    sync();
    return gather();
  }
};
