// Wave-cooperative Fp for the latency path's exponentiation chains (gfx950).
//
// One Fp value per wavefront: limb l (28-bit, Montgomery form, the fp_t limb) in lane l for
// l < 14, and 0 in lanes 14..63.  A product spreads the 392 multiply-adds of fp_mul_body over
// the lanes so that one lane's chain is ~30 v_mad_u64_u32 instead of 392: the single-lane
// exponentiations of the small calls (SSWU, signature decompression; ~460 dependent products
// each, ~0.9 us per product on one lane) are latency chains with the rest of the chip idle.
//
// Product layout (column c of the 28-column product sum lives in lane (c - 14) mod 64):
//   the result columns 14..27 land in lanes 0..13, the home lanes of the operands, and the
//   low columns 0..13, consumed one per reduction row, in lanes 50..63.
//   a.b:  lane L accumulates a_i * b_{c(L) - i} over i; the b operand rotated by 14 - i
//         (DPP wave_rol:1 steps; lanes 14..63 of b are 0, so out-of-range terms read 0).
//   rows: for i = 0..13, column i (lane 50 + i) read to scalars with the running carry,
//         m_i = (col_i + carry) n0 mod 2^28 on the scalar unit, and every lane adds
//         m_i * p_{c(L) - i} (p rotated the same way, per wave constants).
//   out:  the carry of row 13 into column 14, two parallel carry passes (DPP wave_shr:1):
//         limbs < 2^28 + 2^8 (fp_mul accepts < 2^29), value (ab + mp) / R as fp_mul_body.
// Column bound: 14 a.b and 14 m.p terms of < 2^58 each, < 2^62.9, plus carries < 2^36.
#pragma once
#include "bls_field.h"

#if defined(__HIPCC__)

// N' = -p^-1 mod 2^392 (28-bit limbs; limb 0 is BGV_N0), for the lane-parallel reduction
#define BGV_NPRIME_LIMBS                                                                              \
  {0xffcfffdu, 0xf3fffcfu, 0x113e889u, 0xdb92d9du, 0xb48286au, 0xf0c8e30u, 0xc16ef2eu, 0x8eb2db4u, \
   0x9ecca0eu, 0x68cf581u, 0x316fee2u, 0xfc9468bu, 0x106feaau, 0xa0ceb06u}

struct wfp_ctx {
  uint32_t lane;
  uint32_t prot[NL];  // prot[i]: p's limb c(L) - i in lane L (0 outside 0..13)
  uint32_t nrot[NL];  // nrot[i]: N''s limb c(L) - i in lane L (0 outside 0..13)
};

__device__ __forceinline__ uint32_t wfp_lane() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// lane L reads lane (L + 1) mod 64 (DPP wave_rol:1)
__device__ __forceinline__ uint32_t wfp_rol1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xf, 0xf, false);
}

// lane L reads lane (L - 1) mod 64 (DPP wave_ror:1)
__device__ __forceinline__ uint32_t wfp_ror1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13c, 0xf, 0xf, false);
}

// lane L reads lane L - 1 (DPP wave_shr:1); lane 0 reads 0
__device__ __forceinline__ uint32_t wfp_shr1(uint32_t v, uint32_t lane) {
  const uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
  return lane == 0 ? 0u : x;
}

__device__ __forceinline__ wfp_ctx wfp_init() {
  wfp_ctx c;
  c.lane = wfp_lane();
  uint32_t r = 0;
  BGV_UNROLL for (int l = 0; l < NL; ++l) r = c.lane == (uint32_t)l ? p_limb(l) : r;
  BGV_UNROLL for (int k = 1; k <= NL; ++k) {
    r = wfp_rol1(r);
    c.prot[NL - k] = r;
  }
  const uint32_t NP[NL] = BGV_NPRIME_LIMBS;
  r = 0;
  BGV_UNROLL for (int l = 0; l < NL; ++l) r = c.lane == (uint32_t)l ? NP[l] : r;
  BGV_UNROLL for (int k = 1; k <= NL; ++k) {
    r = wfp_rol1(r);
    c.nrot[NL - k] = r;
  }
  return c;
}

// a wave-uniform fp_t -> one limb per lane
__device__ __forceinline__ uint32_t wfp_from(const fp_t& x, const wfp_ctx& c) {
  uint32_t r = 0;
  BGV_UNROLL for (int l = 0; l < NL; ++l) r = c.lane == (uint32_t)l ? x.v[l] : r;
  return r;
}

// one limb per lane -> a wave-uniform fp_t with normalized limbs (same value)
__device__ __forceinline__ fp_t wfp_to(uint32_t v) {
  fp_t r;
  uint32_t carry = 0;
  BGV_UNROLL for (int l = 0; l < NL - 1; ++l) {
    const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)v, l) + carry;
    r.v[l] = s & LMASK;
    carry = s >> LBITS;
  }
  r.v[NL - 1] = (uint32_t)__builtin_amdgcn_readlane((int)v, NL - 1) + carry;
  return r;
}

// (a b + m p) / 2^392 with one limb per lane; operand limbs < 2^29, values as fp_mul's.
// K: reduction columns per scalar round (the m digits of K columns computed on the scalar
// unit from one batch of column reads, with the cross terms m_j p_(c-j) inside the batch
// added there), so the column-read -> scalar -> multiply-add round trip happens ceil(14/K)
// times.  ACC: independent accumulators of the a.b phase (chain depth 14 / ACC).
template <int K, int ACC>
__device__ __forceinline__ uint32_t wfp_mul_t(uint32_t a, uint32_t b, const wfp_ctx& c) {
  uint32_t br[NL];
  uint32_t r = b;
  BGV_UNROLL for (int k = 1; k <= NL; ++k) {
    r = wfp_rol1(r);
    br[NL - k] = r;
  }
  uint64_t acc[ACC];
  BGV_UNROLL for (int q = 0; q < ACC; ++q) acc[q] = 0;
  BGV_UNROLL for (int i = NL - 1; i >= 0; --i)
    acc[i % ACC] += (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)a, i) * br[i];
  uint64_t col = acc[0];
  BGV_UNROLL for (int q = 1; q < ACC; ++q) col += acc[q];
  uint64_t carry = 0;
  BGV_UNROLL for (int i0 = 0; i0 < NL; i0 += K) {
    constexpr int KK = K;
    uint64_t x[KK];
    uint32_t m[KK];
    BGV_UNROLL for (int j = 0; j < KK; ++j) {
      if (i0 + j >= NL) break;
      const uint32_t xl = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)col, 50 + i0 + j);
      const uint32_t xh = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(col >> 32), 50 + i0 + j);
      x[j] = ((uint64_t)xh << 32) | xl;
    }
    BGV_UNROLL for (int j = 0; j < KK; ++j) {
      if (i0 + j >= NL) break;
      uint64_t s = x[j] + carry;
      BGV_UNROLL for (int jj = 0; jj < j; ++jj) s += (uint64_t)m[jj] * p_limb(j - jj);
      m[j] = ((uint32_t)s * BGV_N0) & LMASK;
      carry = (s + (uint64_t)m[j] * p_limb(0)) >> LBITS;
    }
    BGV_UNROLL for (int j = 0; j < KK; ++j) {
      if (i0 + j >= NL) break;
      col += (uint64_t)m[j] * c.prot[i0 + j];
    }
  }
  const uint64_t v = col + (c.lane == 0 ? carry : 0);
  const uint32_t lo = (uint32_t)v & LMASK;
  const uint64_t hi = v >> LBITS;
  const uint64_t hs = ((uint64_t)wfp_shr1((uint32_t)(hi >> 32), c.lane) << 32) | wfp_shr1((uint32_t)hi, c.lane);
  const uint64_t v1 = lo + hs;
  const uint32_t res = ((uint32_t)v1 & LMASK) + wfp_shr1((uint32_t)(v1 >> LBITS), c.lane);
  return c.lane < NL ? res : 0u;
}

// The same product with the reduction as two more lane-parallel products instead of 14
// scalar rounds (one wave issues at most one instruction per 4 cycles, so the chain's
// instruction count is its latency):
//   T = a b (28 columns);  t = T mod R, limbs < 2^29 (two carry passes on a copy, the carry
//   out of column 13 dropped);  m = t N' mod R (columns 0..13 of the product, two carry
//   passes, limbs < 2^29);  U = T + m p.  U's low half is 0 mod R with redundant limbs: after
//   two carry passes over the whole ring (lane 63 -> lane 0) its limbs are < 2^28 + 2^9 and
//   sum to 0 or exactly R, i.e. R iff some low limb is nonzero (a ballot).  m may exceed R by
//   its redundancy (< R (1 + 2^-19)); the result stays below 2p.
__device__ __forceinline__ uint32_t wfp_mul3(uint32_t a, uint32_t b, const wfp_ctx& c) {
  uint32_t br[NL];
  uint32_t r = b;
  BGV_UNROLL for (int k = 1; k <= NL; ++k) {
    r = wfp_rol1(r);
    br[NL - k] = r;
  }
  uint64_t T = 0;
  BGV_UNROLL for (int i = NL - 1; i >= 0; --i) T += (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)a, i) * br[i];
  // t = T mod R (lanes 50..63; lanes 14..49 stay 0, so lane 50 receives no carry)
  uint32_t t;
  {
    const uint64_t h = T >> LBITS;
    const uint64_t v1 = (uint64_t)((uint32_t)T & LMASK) +
                        (((uint64_t)wfp_shr1((uint32_t)(h >> 32), c.lane) << 32) | wfp_shr1((uint32_t)h, c.lane));
    t = ((uint32_t)v1 & LMASK) + wfp_shr1((uint32_t)(v1 >> LBITS), c.lane);
  }
  uint64_t M = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) M += (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)t, 50 + i) * c.nrot[i];
  uint32_t m;
  {
    const uint64_t h = M >> LBITS;
    const uint64_t v1 = (uint64_t)((uint32_t)M & LMASK) +
                        (((uint64_t)wfp_shr1((uint32_t)(h >> 32), c.lane) << 32) | wfp_shr1((uint32_t)h, c.lane));
    m = ((uint32_t)v1 & LMASK) + wfp_shr1((uint32_t)(v1 >> LBITS), c.lane);
  }
  BGV_UNROLL for (int i = 0; i < NL; ++i) T += (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)m, 50 + i) * c.prot[i];
  const uint64_t h = T >> LBITS;
  const uint64_t v1 = (uint64_t)((uint32_t)T & LMASK) + (((uint64_t)wfp_ror1((uint32_t)(h >> 32)) << 32) | wfp_ror1((uint32_t)h));
  const uint32_t v2 = ((uint32_t)v1 & LMASK) + wfp_ror1((uint32_t)(v1 >> LBITS));
  const uint64_t low = __ballot(v2 != 0) & 0xFFFC000000000000ull;  // lanes 50..63
  const uint32_t res = v2 + (c.lane == 0 && low != 0 ? 1u : 0u);
  return c.lane < NL ? res : 0u;
}

// A product of two WAVE-UNIFORM fp_t values (every lane holds the same a and b) on the whole
// wave, returning the uniform product (normalized limbs): the drop-in for fp_mul in code that
// runs one set per wave.  Same three lane-parallel products as wfp_mul3, arranged so that no
// per-wave constants are needed: a.b takes a's limbs straight from the (uniform) VGPRs and b
// rotated; t N' and m p take N' and p as scalar constants and rotate t and m instead (lane L
// reads lane L - j: wave_ror steps; t and m are masked to lanes 50..63, so terms outside a
// column's range read 0).  The value equals fp_mul_body's: (ab + mp) / R with m = -ab/p mod R.
// (limbs as 28 scalar arguments, as fp_mul_l: a second struct argument would travel through
// scratch memory on every call)
__device__ __noinline__ fp_t wfp_umul_l(BGV_U14(a_), BGV_U14(b_)) {
  const fp_t a = {{BGV_L14(a_)}}, b = {{BGV_L14(b_)}};
  const uint32_t lane = wfp_lane();
  const bool low = lane >= 50;
  uint32_t r = 0;
  BGV_UNROLL for (int l = 0; l < NL; ++l) r = lane == (uint32_t)l ? b.v[l] : r;
  uint32_t br[NL];
  BGV_UNROLL for (int k = 1; k <= NL; ++k) {
    r = wfp_rol1(r);
    br[NL - k] = r;
  }
  uint64_t T = 0;
  BGV_UNROLL for (int i = NL - 1; i >= 0; --i) T += (uint64_t)a.v[i] * br[i];
  // t = T mod R in lanes 50..63 (0 elsewhere)
  uint32_t t;
  {
    const uint64_t h = T >> LBITS;
    const uint64_t v1 = (uint64_t)((uint32_t)T & LMASK) +
                        (((uint64_t)wfp_shr1((uint32_t)(h >> 32), lane) << 32) | wfp_shr1((uint32_t)h, lane));
    t = ((uint32_t)v1 & LMASK) + wfp_shr1((uint32_t)(v1 >> LBITS), lane);
    t = low ? t : 0u;
  }
  const uint32_t NP[NL] = BGV_NPRIME_LIMBS;
  uint64_t M = (uint64_t)NP[0] * t;
  uint32_t tr = t;
  BGV_UNROLL for (int j = 1; j < NL; ++j) {
    tr = wfp_ror1(tr);
    M += (uint64_t)NP[j] * tr;
  }
  uint32_t m;
  {
    const uint64_t h = M >> LBITS;
    const uint64_t v1 = (uint64_t)((uint32_t)M & LMASK) +
                        (((uint64_t)wfp_shr1((uint32_t)(h >> 32), lane) << 32) | wfp_shr1((uint32_t)h, lane));
    m = ((uint32_t)v1 & LMASK) + wfp_shr1((uint32_t)(v1 >> LBITS), lane);
    m = low ? m : 0u;
  }
  uint32_t mr = m;
  T += (uint64_t)p_limb(0) * mr;
  BGV_UNROLL for (int j = 1; j < NL; ++j) {
    mr = wfp_ror1(mr);
    T += (uint64_t)p_limb(j) * mr;
  }
  const uint64_t h = T >> LBITS;
  const uint64_t v1 = (uint64_t)((uint32_t)T & LMASK) + (((uint64_t)wfp_ror1((uint32_t)(h >> 32)) << 32) | wfp_ror1((uint32_t)h));
  const uint32_t v2 = ((uint32_t)v1 & LMASK) + wfp_ror1((uint32_t)(v1 >> LBITS));
  const uint64_t lowbits = __ballot(v2 != 0) & 0xFFFC000000000000ull;
  const uint32_t res = v2 + (lane == 0 && lowbits != 0 ? 1u : 0u);
  return wfp_to(res);
}
__device__ __forceinline__ fp_t wfp_umul(const fp_t& a, const fp_t& b) { return wfp_umul_l(BGV_V14(a), BGV_V14(b)); }

#ifndef BGV_WFP_K
#define BGV_WFP_K 2
#endif
#ifndef BGV_WFP_ACC
#define BGV_WFP_ACC 2
#endif
__device__ __forceinline__ uint32_t wfp_mul(uint32_t a, uint32_t b, const wfp_ctx& c) {
#ifdef BGV_WFP_ROWS
  return wfp_mul_t<BGV_WFP_K, BGV_WFP_ACC>(a, b, c);
#else
  return wfp_mul3(a, b, c);
#endif
}

// a^e for kBgvPow[W]'s exponent on the whole wave (every lane calls it with the same a, in
// uniform control flow); the same window schedule as fp_pow_fixed, so the same value.
template <int W>
__device__ __noinline__ fp_t wfp_pow_fixed(const fp_t& a_u) {
  const wfp_ctx c = wfp_init();
  const bgv_pow_sched& s = kBgvPow[W];
  const uint32_t a = wfp_from(a_u, c);
  uint32_t tab[16];
  tab[0] = a;
  const uint32_t a2 = wfp_mul(a, a, c);
  uint32_t cur = a;
  BGV_NO_UNROLL for (int k = 1; k < 16; ++k) {
    cur = wfp_mul(cur, a2, c);
    tab[k] = cur;
  }
  uint32_t r = tab[s.first];
  BGV_NO_UNROLL for (int k = 0; k < s.n; ++k) {
    const uint32_t st = s.step[k];
    const int d = (int)(st >> 8), nsq = (int)(st & 0xff);
    const uint32_t m = tab[d & 15];
    BGV_NO_UNROLL for (int q = 0; q < nsq; ++q) r = wfp_mul(r, r, c);
    if (d != 0xff) r = wfp_mul(r, m, c);
  }
  return wfp_to(r);
}

// The exponentiation policy of the square roots (bls_field.h bgv_pow_lane) on the wavefront:
// for code that runs one set per wave with every lane holding the same values.
struct bgv_pow_wave {
  static __device__ fp_t p34(const fp_t& a) { return wfp_pow_fixed<BGV_POW_P34>(a); }
  static __device__ fp_t sqrt_exp(const fp_t& a) { return wfp_pow_fixed<BGV_POW_SQRT>(a); }
};

#endif  // __HIPCC__
