// Deferred (double-width) reduction for the per-lane Fp2 products (gfx950, one element per lane).
//
// blst's Fp2 product (mul_mont_384x) is Karatsuba with the reduction deferred: three
// double-width products t0 = a0 b0, t1 = a1 b1, t2 = (a0 + a1)(b0 + b1), then ONE Montgomery
// reduction per output coefficient, c0 = REDC(t0 - t1) and c1 = REDC(t2 - t0 - t1): 3 products
// + 2 reductions (980 v_mad_u64_u32 with 28-bit limbs) against 3 fully reduced products (1,176).
// On a CPU the double-width values sit in memory; one lane cannot hold three 27-column
// products (54 VGPRs each), so the product here is the finely integrated product-scanning
// form: column k of t0, t1 and t2 is summed, combined into column k of the two double-width
// values D = t0 - t1 and S = t2 - t0 - t1, and each of D and S runs its own reduction row in
// the same column.  Between columns the only state is two carries and the 2 x 14 reduction
// digits m_i, so nothing double-width is ever stored.
//
//   * No stream is ever negative: t1 enters both outputs through the negated operand
//     b1n = k p - b1 (a redundant k p whose limbs cover b1's bound, lzc::make_kp), so
//     t1' = a1 b1n = k p a1 - a1 b1 and D = t0 + t1', S = t2 - t0 + t1' agree with the
//     Karatsuba coefficients mod p.  Column by column D and S are sums of non-negative
//     products (S_k = sum a0_i b1_j + a1_i b0_j + a1_i kp_j), so both streams are unsigned;
//     intermediate wrap-around of t2 - t0 is harmless, only each column's final value must fit
//     (bgvw::mul_ok, asserted at every use in bls_lazy.h).
//   * Values: D < (VA VB + VA k) p^2 and S < (2 VA VB + VA k) p^2, so both results stay
//     below 2p when those sums are <= 2520 = floor(R / p) (below 3p up to 5040).
//
// The out-of-line products take a (the 28 limbs of a0, a1) in VGPR arguments; the AMDGPU
// calling convention passes at most 32 VGPRs and returns a struct of more than 16 dwords
// through scratch, so b waits in a per-lane LDS slot (bgv_wslot, 7 x 16 B per lane, written
// by the caller just before the call) and the 28-limb result returns as a 28-element vector in
// VGPRs.  The slot is indexed by the lane id: units that use these products (BGV_LZ2_WIDE,
// bgv_k_prep_bulk.hip / bgv_k_miller_bulk.hip) launch one-wave (64-thread) blocks only.
#pragma once
#include <utility>

#include "bls_field.h"

#if defined(__clang__)
typedef uint32_t bgv_u28 __attribute__((ext_vector_type(28)));
#else
struct bgv_u28 {
  uint32_t e[28];
  uint32_t& operator[](int i) { return e[i]; }
  uint32_t operator[](int i) const { return e[i]; }
};
#endif

// ---------------------------------------------------------------------------------------------
// the per-lane operand slot
// ---------------------------------------------------------------------------------------------
#if defined(__HIP_DEVICE_COMPILE__)
static __shared__ uint4 bgv_wslot[7][64];
__device__ __forceinline__ void wslot_put(const uint32_t* w, int n) {  // n words, n % 4 == 0 or n == 14
  const uint32_t l = __lane_id();
  BGV_UNROLL for (int q = 0; q < (n + 3) / 4; ++q) {
    const int b = 4 * q;
    bgv_wslot[q][l] = make_uint4(w[b], b + 1 < n ? w[b + 1] : 0u, b + 2 < n ? w[b + 2] : 0u, b + 3 < n ? w[b + 3] : 0u);
  }
}
__device__ __forceinline__ void wslot_get(uint32_t* w, int n) {
  const uint32_t l = __lane_id();
  BGV_UNROLL for (int q = 0; q < (n + 3) / 4; ++q) {
    const uint4 v = bgv_wslot[q][l];
    const int b = 4 * q;
    w[b] = v.x;
    if (b + 1 < n) w[b + 1] = v.y;
    if (b + 2 < n) w[b + 2] = v.z;
    if (b + 3 < n) w[b + 3] = v.w;
  }
}
#else
static thread_local uint32_t bgv_wslot_h[28];
inline void wslot_put(const uint32_t* w, int n) {
  for (int i = 0; i < n; ++i) bgv_wslot_h[i] = w[i];
}
inline void wslot_get(uint32_t* w, int n) {
  for (int i = 0; i < n; ++i) w[i] = bgv_wslot_h[i];
}
#endif

// ---------------------------------------------------------------------------------------------
// bodies (also the host reference: tests/native/hostsim.cpp)
// ---------------------------------------------------------------------------------------------
// The slot operand's negation b1n = KM - b1 and the squaring's a0 - a1 + KS: fixed redundant
// multiples of p for the operand bounds the out-of-line entries accept.
#define BGV_WMUL_LB ((1ull << 29) - 1)
#define BGV_WMUL_VB 8
#define BGV_WSQR_LIMB ((1ull << 28) + (1ull << 27))
#define BGV_WSQR_V 8
namespace bgvw {
constexpr lzc::kp KM = lzc::make_kp(BGV_WMUL_LB, BGV_WMUL_VB);
constexpr lzc::kp KS = lzc::make_kp(BGV_WSQR_LIMB, BGV_WSQR_V);
static_assert(KM.k != 0 && KS.k != 0, "bls_wide: no k p representation");
constexpr uint64_t PMAX = 0xfffffffull;  // largest limb of p
typedef unsigned __int128 u128;
// the largest final column value of a stream whose operand products sum to at most sum_ab per
// column, plus its 14 reduction terms m_i p_j and the carry in
constexpr u128 col_max(u128 sum_ab) { return sum_ab + (u128)14 * LMASK * PMAX + ((u128)1 << 37); }
constexpr u128 TWO64 = (u128)1 << 64;
// fp2_mul_w_body for a limbs <= la and b limbs <= lb (b in the slot)
constexpr bool mul_ok(uint64_t la, uint64_t lb) {
  return lb <= BGV_WMUL_LB && 2 * la <= 0xffffffffull &&
         col_max((u128)14 * la * (2 * lb + KM.maxl)) < TWO64 &&  // S
         col_max((u128)14 * la * (lb + KM.maxl)) < TWO64;        // D
}
// the value bound (in p) of both results for operand values va, vb (b in the slot): 0 if too big
constexpr uint64_t mul_vout(uint64_t va, uint64_t vb) {
  const uint64_t m = 2 * va * vb + va * KM.k;
  return vb > BGV_WMUL_VB ? 0 : (m <= 2520 ? 2 : (m <= 5040 ? 3 : 0));
}
// fp_mul2_w_body for x, z limbs <= lx and y, w limbs <= ly
constexpr bool mul2_ok(uint64_t lx, uint64_t ly) { return col_max((u128)14 * lx * ly) < TWO64; }
static_assert(mul2_ok(2 * BGV_WSQR_LIMB, BGV_WSQR_LIMB + KS.maxl), "bls_wide: squaring column sums overflow");
static_assert(2 * BGV_WSQR_V * (BGV_WSQR_V + KS.k) < 2520, "bls_wide: squaring value bound");

// The column loops are compile-time recursions (one instantiation per column k), so every
// index is a constant and nothing is indexed dynamically: a plain `#pragma unroll` over 27
// columns with triangular inner loops was left rolled by the compiler (VGPR-indexed arrays).
struct mul_state {
  uint32_t sa[NL], sb[NL], md[NL], ms[NL];
  uint64_t cd, cs;
};
template <int K>
BGV_HD void mul_col(mul_state& st, const uint32_t* a0, const uint32_t* a1, const uint32_t* b0, const uint32_t* b1n,
                    uint32_t* r0, uint32_t* r1) {
  const uint32_t P_[NL] = BGV_P_LIMBS;
  // the column's product sums and its reduction terms from the earlier digits do not depend on
  // the carry in, so they are summed from 0 and the carry joins last: the serial path from one
  // column to the next is the carry, one digit and its two terms, not the whole column
  uint64_t e = 0, q = 0, s = 0, dm = 0, sm = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    const int j = K - i;
    if (j < 0 || j >= NL) continue;
    e += (uint64_t)a0[i] * b0[j];
    q += (uint64_t)a1[i] * b1n[j];
    s += (uint64_t)st.sa[i] * st.sb[j];
  }
  BGV_UNROLL for (int i = 0; i < NL; ++i) {  // oldest digit first: the newest joins last
    const int j = K - i;
    if (i >= K || j >= NL) continue;
    dm += (uint64_t)st.md[i] * P_[j];
    sm += (uint64_t)st.ms[i] * P_[j];
  }
  uint64_t d = e + q + dm + st.cd;
  s = s - e + q + sm + st.cs;
  if constexpr (K < NL) {
    st.md[K] = ((uint32_t)d * BGV_N0) & LMASK;
    st.ms[K] = ((uint32_t)s * BGV_N0) & LMASK;
    d += (uint64_t)st.md[K] * P_[0];
    s += (uint64_t)st.ms[K] * P_[0];
  } else {
    r0[K - NL] = (uint32_t)d & LMASK;
    r1[K - NL] = (uint32_t)s & LMASK;
  }
  st.cd = d >> LBITS;
  st.cs = s >> LBITS;
}
template <int... K>
BGV_HD void mul_cols(mul_state& st, const uint32_t* a0, const uint32_t* a1, const uint32_t* b0, const uint32_t* b1n,
                     uint32_t* r0, uint32_t* r1, std::integer_sequence<int, K...>) {
  (mul_col<K>(st, a0, a1, b0, b1n, r0, r1), ...);
}

struct mul2_state {
  uint32_t m0[NL], m1[NL];
  uint64_t c0, c1;
};
template <int K>
BGV_HD void mul2_col(mul2_state& st, const uint32_t* x, const uint32_t* y, const uint32_t* z, const uint32_t* w,
                     uint32_t* r0, uint32_t* r1) {
  const uint32_t P_[NL] = BGV_P_LIMBS;
  uint64_t u = 0, v = 0, um = 0, vm = 0;  // the carry joins last (see mul_col)
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    const int j = K - i;
    if (j < 0 || j >= NL) continue;
    u += (uint64_t)x[i] * y[j];
    v += (uint64_t)z[i] * w[j];
  }
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    const int j = K - i;
    if (i >= K || j >= NL) continue;
    um += (uint64_t)st.m0[i] * P_[j];
    vm += (uint64_t)st.m1[i] * P_[j];
  }
  u = u + um + st.c0;
  v = v + vm + st.c1;
  if constexpr (K < NL) {
    st.m0[K] = ((uint32_t)u * BGV_N0) & LMASK;
    st.m1[K] = ((uint32_t)v * BGV_N0) & LMASK;
    u += (uint64_t)st.m0[K] * P_[0];
    v += (uint64_t)st.m1[K] * P_[0];
  } else {
    r0[K - NL] = (uint32_t)u & LMASK;
    r1[K - NL] = (uint32_t)v & LMASK;
  }
  st.c0 = u >> LBITS;
  st.c1 = v >> LBITS;
}
template <int... K>
BGV_HD void mul2_cols(mul2_state& st, const uint32_t* x, const uint32_t* y, const uint32_t* z, const uint32_t* w,
                      uint32_t* r0, uint32_t* r1, std::integer_sequence<int, K...>) {
  (mul2_col<K>(st, x, y, z, w, r0, r1), ...);
}
}  // namespace bgvw

// r0 = REDC(a0 b0 + a1 (KM - b1)) = a0 b0 - a1 b1, r1 = REDC((a0 + a1)(b0 + b1) - a0 b0 + a1 (KM - b1))
// = a0 b1 + a1 b0 (mod p); limbs 0..12 of each < 2^28, limb 13 the top carry.
BGV_HD void fp2_mul_w_body(const uint32_t* a0, const uint32_t* a1, const uint32_t* b0, const uint32_t* b1,
                           uint32_t* r0, uint32_t* r1) {
  bgvw::mul_state st;
  uint32_t b1n[NL];
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    st.sa[i] = a0[i] + a1[i];
    st.sb[i] = b0[i] + b1[i];
    b1n[i] = bgvw::KM.v[i] - b1[i];
  }
  st.cd = st.cs = 0;
  bgvw::mul_cols(st, a0, a1, b0, b1n, r0, r1, std::make_integer_sequence<int, 2 * NL - 1>{});
  r0[NL - 1] = (uint32_t)st.cd;
  r1[NL - 1] = (uint32_t)st.cs;
}

// Two independent reductions side by side: r0 = REDC(x y), r1 = REDC(z w) (unsigned streams).
// The squaring (x = a0 + a1, y = a0 - a1 + k p, z = 2 a0, w = a1) and the Fp2-by-Fp product
// (x = a0, z = a1, y = w = s) are this with their operands formed by the caller of the body.
BGV_HD void fp_mul2_w_body(const uint32_t* x, const uint32_t* y, const uint32_t* z, const uint32_t* w,
                           uint32_t* r0, uint32_t* r1) {
  bgvw::mul2_state st;
  st.c0 = st.c1 = 0;
  bgvw::mul2_cols(st, x, y, z, w, r0, r1, std::make_integer_sequence<int, 2 * NL - 1>{});
  r0[NL - 1] = (uint32_t)st.c0;
  r1[NL - 1] = (uint32_t)st.c1;
}

// (a0 + a1)(a0 - a1 + KS), (2 a0) a1 for limbs <= BGV_WSQR_LIMB, values < BGV_WSQR_V p
BGV_HD void fp2_sqr_w_body(const uint32_t* a0, const uint32_t* a1, uint32_t* r0, uint32_t* r1) {
  uint32_t x[NL], y[NL], z[NL];
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    x[i] = a0[i] + a1[i];
    y[i] = a0[i] + (bgvw::KS.v[i] - a1[i]);
    z[i] = a0[i] + a0[i];
  }
  fp_mul2_w_body(x, y, z, a1, r0, r1);
}

// ---------------------------------------------------------------------------------------------
// out-of-line entries: a0, a1 in VGPR arguments, the other operand from the lane's slot
// ---------------------------------------------------------------------------------------------
BGV_HD bgv_u28 w28_pack(const uint32_t* r0, const uint32_t* r1) {
  bgv_u28 o;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    o[i] = r0[i];
    o[NL + i] = r1[i];
  }
  return o;
}

// Fp2 product: b0 | b1 in the slot (28 words)
BGV_MUL_ATTR bgv_u28 fp2_mul_w_l(BGV_U14(a0_), BGV_U14(a1_)) {
  BGV_COUNT_MUL();
  BGV_COUNT_MUL();
  BGV_COUNT_MUL();
  const uint32_t a0[NL] = {BGV_L14(a0_)}, a1[NL] = {BGV_L14(a1_)};
  uint32_t b[2 * NL], r0[NL], r1[NL];
  wslot_get(b, 2 * NL);
  fp2_mul_w_body(a0, a1, b, b + NL, r0, r1);
  return w28_pack(r0, r1);
}

// Fp2 by Fp: s in the slot (14 words)
BGV_MUL_ATTR bgv_u28 fp2_mul_fp_w_l(BGV_U14(a0_), BGV_U14(a1_)) {
  BGV_COUNT_MUL();
  BGV_COUNT_MUL();
  const uint32_t a0[NL] = {BGV_L14(a0_)}, a1[NL] = {BGV_L14(a1_)};
  uint32_t s[NL], r0[NL], r1[NL];
  wslot_get(s, NL);
  fp_mul2_w_body(a0, s, a1, s, r0, r1);
  return w28_pack(r0, r1);
}

// Fp2 square: no slot (operand bounds BGV_WSQR_LIMB / BGV_WSQR_V, checked by the caller)
BGV_MUL_ATTR bgv_u28 fp2_sqr_w_l(BGV_U14(a0_), BGV_U14(a1_)) {
  BGV_COUNT_SQR();
  BGV_COUNT_SQR();
  const uint32_t a0[NL] = {BGV_L14(a0_)}, a1[NL] = {BGV_L14(a1_)};
  uint32_t r0[NL], r1[NL];
  fp2_sqr_w_body(a0, a1, r0, r1);
  return w28_pack(r0, r1);
}
