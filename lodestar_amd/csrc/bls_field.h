// BLS12-381 field tower for CDNA4 (gfx950): Fp, Fp2, Fp6, Fp12.
//
// One field element per lane.  Fp is stored as 14 unsaturated 28-bit limbs
// (one per u32, little-endian) in Montgomery form with R = 2^392.  Measured
// on MI355X (tools/ubench_fpmul.hip): the row-wise 28-bit Montgomery product
// lowers to 392 independent v_mad_u64_u32 with 64-bit accumulators and no
// carry chains, and runs 1.7x faster than 12 x 32-bit CIOS (whose carries the
// compiler splits into v_mov/v_lshl_add_u64 pairs).  v_mad_u64_u32 issues at
// half rate (16 lanes/clk/SIMD), so the 28-bit product is mad-bound.
//
// Value invariant ("weakly reduced"): every fp_t holds normalized limbs
// (< 2^28) and a value in [0, 2p).  fp_mul accepts inputs up to 4p with limbs
// up to 2^29 (so a + b of two reduced values may feed it directly through
// fp_add_nr) and returns a weakly reduced value: (ab + mp)/R < 16p^2/R + p < 2p.
// Only comparisons and serialisation canonicalise to [0, p).
//
// Tower (same as blst / the IETF pairing draft):
//   Fp2  = Fp[i]  / (i^2 + 1)
//   Fp6  = Fp2[v] / (v^3 - (1 + i))
//   Fp12 = Fp6[w] / (w^2 - v)
//
// The same source compiles for the host (tests/hostsim) so every formula is
// unit-tested against oracle/bls12381.py on the CPU before it runs on a GPU.
#pragma once
#include <stdint.h>

#include "bls_constants.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BGV_HD __host__ __device__ __forceinline__
// static: every kernel unit (bgv_k_*.hip) carries its own copy (no device linking; the
// host-side copies must not collide at link time either)
#define BGV_NOINLINE static __host__ __device__ __noinline__
#else
#define BGV_HD inline __attribute__((always_inline))
#define BGV_NOINLINE __attribute__((noinline))
#endif

// The Montgomery product is the only out-of-line primitive: ~560 instructions
// per call, so the call is cheap, and keeping it out of line keeps kernels small
// enough to compile in seconds rather than hours.
#ifndef BGV_MUL_ATTR
#define BGV_MUL_ATTR BGV_NOINLINE
#endif

// The tower functions of the Miller-loop step (fp6_mul, fp6_mul_01, fp12_sqr, the
// line products, miller_dbl/add) are inlined into their callers, so f, T and the
// lines stay in VGPRs and only fp_mul/fp_sqr are calls: out of line, every
// by-reference argument and struct return went through scratch, and at one wave
// per SIMD nothing hid that latency (k_miller 51.4 -> 41.3 ms per 131,072 sets).
#define BGV_MILLER_ATTR BGV_HD

#define BGV_UNROLL _Pragma("unroll")
#define BGV_NO_UNROLL _Pragma("unroll 1")

// Host-only op counting (tools/count_ops.py builds tests/native/hostsim.cpp with
// -DBGV_COUNT_OPS to count Fp products per kernel for the roofline accounting).
#if defined(BGV_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
extern "C" unsigned long long bgv_count_mul, bgv_count_sqr;
#define BGV_COUNT_MUL() (++bgv_count_mul)
#define BGV_COUNT_SQR() (++bgv_count_sqr)
#else
#define BGV_COUNT_MUL() ((void)0)
#define BGV_COUNT_SQR() ((void)0)
#endif

#define NL 14
#define LBITS 28
#define LMASK 0x0fffffffu

struct fp_t {
  uint32_t v[NL];
};
struct fp2_t {
  fp_t c0, c1;
};
struct fp6_t {
  fp2_t c0, c1, c2;
};
struct fp12_t {
  fp6_t c0, c1;
};

// ---------------------------------------------------------------------------
// Fp
// ---------------------------------------------------------------------------
BGV_HD uint32_t p_limb(int i) {
  const uint32_t P_[NL] = BGV_P_LIMBS;
  return P_[i];
}
BGV_HD uint32_t p2_limb(int i) {
  const uint32_t P_[NL] = BGV_2P_LIMBS;
  return P_[i];
}

BGV_HD fp_t fp_zero() {
  fp_t r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = 0;
  return r;
}

BGV_HD fp_t fp_one() {
  fp_t r = {BGV_ONE};
  return r;
}

// r = cond ? b : a   (branch-free select)
BGV_HD fp_t fp_select(bool cond, const fp_t& a, const fp_t& b) {
  fp_t r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = cond ? b.v[i] : a.v[i];
  return r;
}

// a - 2p when a >= 2p (a normalized, a < 4p); result in [0, 2p).
BGV_HD fp_t fp_reduce_2p(const fp_t& a) {
  fp_t d;
  int32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)a.v[i] - (int32_t)p2_limb(i) + c;
    d.v[i] = (uint32_t)s & LMASK;
    c = s >> LBITS;  // arithmetic: -1 or 0
  }
  return fp_select(c < 0, d, a);
}

// plain limb-wise sum, no carry and no reduction: only as an fp_mul/fp_sqr
// operand (limbs < 2^29, value < 4p)
BGV_HD fp_t fp_add_nr(const fp_t& a, const fp_t& b) {
  fp_t r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}

// a + b with the carries propagated and no reduction: normalized limbs (< 2^28),
// value < A + B.  For Karatsuba operand sums that only ever feed a product.
BGV_HD fp_t fp_add_norm(const fp_t& a, const fp_t& b) {
  fp_t r;
  uint32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    const uint32_t s = a.v[i] + b.v[i] + c;
    r.v[i] = s & LMASK;
    c = s >> LBITS;
  }
  return r;
}

BGV_HD fp_t fp_add(const fp_t& a, const fp_t& b) {
  fp_t r;
  uint32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    uint32_t s = a.v[i] + b.v[i] + c;
    r.v[i] = s & LMASK;
    c = s >> LBITS;
  }
  return fp_reduce_2p(r);
}

BGV_HD fp_t fp_dbl(const fp_t& a) { return fp_add(a, a); }

// a - b + 2p, normalized, in (0, 4p): only as an fp_mul operand
BGV_HD fp_t fp_sub_nr(const fp_t& a, const fp_t& b) {
  fp_t r;
  int32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)a.v[i] - (int32_t)b.v[i] + (int32_t)p2_limb(i) + c;
    r.v[i] = (uint32_t)s & LMASK;
    c = s >> LBITS;
  }
  return r;
}

BGV_HD fp_t fp_sub(const fp_t& a, const fp_t& b) {
  // d = a - b; if negative add 2p
  fp_t d, r;
  int32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)a.v[i] - (int32_t)b.v[i] + c;
    d.v[i] = (uint32_t)s & LMASK;
    c = s >> LBITS;
  }
  const uint32_t m = (uint32_t)c;  // 0 or 0xffffffff
  uint32_t k = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    uint32_t s = d.v[i] + (p2_limb(i) & m) + k;
    r.v[i] = s & LMASK;
    k = s >> LBITS;
  }
  return r;
}

BGV_HD fp_t fp_neg(const fp_t& a) {
  // 2p - a in (0, 2p]; maps 0 to 0 so the result stays below 2p
  fp_t r;
  int32_t c = 0;
  uint32_t nz = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)p2_limb(i) - (int32_t)a.v[i] + c;
    r.v[i] = (uint32_t)s & LMASK;
    c = s >> LBITS;
    nz |= a.v[i];
  }
  return fp_select(nz == 0, r, a);
}

// Montgomery product, row-wise over 28-bit limbs (R = 2^392).  Operand limbs may
// be < 2^29 (an unreduced fp_add_nr): each of the 14 u64 accumulators receives at
// most 2 products per row (< 2^58 + 2^56) over <= 14 rows plus carries, < 2^62.2,
// so no carry ever leaves an accumulator early.  Operand VALUES may be up to 16p
// each: the result is < 256 p^2 / R + p < 1.1 p, weakly reduced.
// The out-of-line products take their limbs as 28 / 14 scalar arguments: the
// AMDGPU calling convention passes those in VGPRs v0..v27, whereas a second
// struct argument would travel through scratch memory on every call.
#define BGV_L14(p) p##0, p##1, p##2, p##3, p##4, p##5, p##6, p##7, p##8, p##9, p##10, p##11, p##12, p##13
#define BGV_U14(p)                                                                                        \
  uint32_t p##0, uint32_t p##1, uint32_t p##2, uint32_t p##3, uint32_t p##4, uint32_t p##5, uint32_t p##6, \
      uint32_t p##7, uint32_t p##8, uint32_t p##9, uint32_t p##10, uint32_t p##11, uint32_t p##12, uint32_t p##13
#define BGV_V14(x) x.v[0], x.v[1], x.v[2], x.v[3], x.v[4], x.v[5], x.v[6], x.v[7], x.v[8], x.v[9], x.v[10], x.v[11], x.v[12], x.v[13]

BGV_HD fp_t fp_mul_body(const fp_t& a, const fp_t& b) {
  const uint32_t P_[NL] = BGV_P_LIMBS;
  uint64_t t[NL];
  BGV_UNROLL for (int j = 0; j < NL; ++j) t[j] = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    BGV_UNROLL for (int j = 0; j < NL; ++j) t[j] += (uint64_t)a.v[i] * b.v[j];
    const uint32_t m = ((uint32_t)t[0] * BGV_N0) & LMASK;
    BGV_UNROLL for (int j = 0; j < NL; ++j) t[j] += (uint64_t)m * P_[j];
    const uint64_t c = t[0] >> LBITS;
    BGV_UNROLL for (int j = 0; j < NL - 1; ++j) t[j] = t[j + 1];
    t[NL - 1] = 0;
    t[0] += c;
  }
  fp_t r;
  BGV_UNROLL for (int j = 0; j < NL - 1; ++j) {
    r.v[j] = (uint32_t)t[j] & LMASK;
    t[j + 1] += t[j] >> LBITS;
  }
  r.v[NL - 1] = (uint32_t)t[NL - 1];
  return r;
}

BGV_MUL_ATTR fp_t fp_mul_l(BGV_U14(a_), BGV_U14(b_)) {
  BGV_COUNT_MUL();
  const fp_t a = {{BGV_L14(a_)}}, b = {{BGV_L14(b_)}};
  return fp_mul_body(a, b);
}

// Montgomery square: 105 products (cross terms doubled) then 14 reduction rows.
BGV_HD fp_t fp_sqr_body(const fp_t& a) {
  const uint32_t P_[NL] = BGV_P_LIMBS;
  uint64_t t[2 * NL];
  BGV_UNROLL for (int j = 0; j < 2 * NL; ++j) t[j] = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    t[2 * i] += (uint64_t)a.v[i] * a.v[i];
    const uint32_t a2 = a.v[i] << 1;
    BGV_UNROLL for (int j = i + 1; j < NL; ++j) t[i + j] += (uint64_t)a2 * a.v[j];
  }
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    const uint32_t m = ((uint32_t)t[i] * BGV_N0) & LMASK;
    BGV_UNROLL for (int j = 0; j < NL; ++j) t[i + j] += (uint64_t)m * P_[j];
    t[i + 1] += t[i] >> LBITS;
  }
  fp_t r;
  BGV_UNROLL for (int j = 0; j < NL - 1; ++j) {
    r.v[j] = (uint32_t)t[NL + j] & LMASK;
    t[NL + j + 1] += t[NL + j] >> LBITS;
  }
  r.v[NL - 1] = (uint32_t)t[2 * NL - 1];
  return r;
}

BGV_MUL_ATTR fp_t fp_sqr_l(BGV_U14(a_)) {
  BGV_COUNT_SQR();
  const fp_t a = {{BGV_L14(a_)}};
  return fp_sqr_body(a);
}

// (A hand-scheduled product subroutine with an exact clobber set, tools/experimental/
// bgv_fpmul_asm.h, measured equal to the ABI call at the kernel level in round 4 and is not
// part of the library.)
#if defined(__HIP_DEVICE_COMPILE__) && defined(BGV_WAVE_UNIFORM_MUL)
// BGV_WAVE_UNIFORM_MUL (device code of a unit whose kernels run one set per wave, every lane
// holding the same values): each product on the whole wave (bgv_wfp.h wfp_umul, defined there).
__device__ __noinline__ fp_t wfp_umul_l(BGV_U14(a_), BGV_U14(b_));
__device__ __forceinline__ fp_t fp_mul(const fp_t& a, const fp_t& b) { return wfp_umul_l(BGV_V14(a), BGV_V14(b)); }
__device__ __forceinline__ fp_t fp_sqr(const fp_t& a) { return wfp_umul_l(BGV_V14(a), BGV_V14(a)); }
#else
BGV_HD fp_t fp_mul(const fp_t& a, const fp_t& b) { return fp_mul_l(BGV_V14(a), BGV_V14(b)); }
BGV_HD fp_t fp_sqr(const fp_t& a) { return fp_sqr_l(BGV_V14(a)); }
#endif

// canonical representative in [0, p) of a weakly reduced value
BGV_HD fp_t fp_canon(const fp_t& a) {
  fp_t d;
  int32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)a.v[i] - (int32_t)p_limb(i) + c;
    d.v[i] = (uint32_t)s & LMASK;
    c = s >> LBITS;
  }
  return fp_select(c < 0, d, a);
}

BGV_HD bool fp_is_zero(const fp_t& a) {
  const fp_t c = fp_canon(a);
  uint32_t acc = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) acc |= c.v[i];
  return acc == 0;
}

BGV_HD bool fp_eq(const fp_t& a, const fp_t& b) { return fp_is_zero(fp_sub(a, b)); }

// to / from Montgomery form (raw integers < 2^392)
BGV_HD fp_t fp_to_mont(const fp_t& a) {
  const fp_t r2 = {BGV_R2};
  return fp_mul(a, r2);
}

// canonical raw integer in [0, p)
BGV_HD fp_t fp_from_mont(const fp_t& a) {
  const fp_t one = {BGV_RAW_ONE};
  return fp_canon(fp_mul(a, one));
}

// a^e for a fixed exponent: left-to-right sliding window of width 5 over a table of the 16
// odd powers a, a^3, ..., a^31.  The exponents used here have ~229 one bits in 381: the
// window cuts the products from ~229 to ~84 (16 of them for the table).  The window
// schedule is computed at compile time (bgv_make_sched) and read from constant memory with
// scalar loads, so the loop does no per-bit exponent reads (these were scratch loads with a
// wait each), and each window's table entry is loaded before its squarings.
struct bgv_exp12 {
  uint32_t w[12];
};
struct bgv_pow_sched {
  int n;                // steps after the first window
  int first;            // r starts as tab[first] = a^(2 first + 1)
  uint32_t step[112];   // step k: (step & 0xff) squarings, then a product by tab[step >> 8]
                        // (0xff: none -- trailing squarings); dwords for scalar loads
};
constexpr int bgv_exp_bit(const bgv_exp12& e, int i) { return (int)((e.w[i >> 5] >> (i & 31)) & 1u); }
constexpr bgv_pow_sched bgv_make_sched(bgv_exp12 e, int nbits) {
  bgv_pow_sched s{};
  bool started = false;
  int pending = 0;
  int i = nbits - 1;
  while (i >= 0) {
    if (!bgv_exp_bit(e, i)) {
      ++pending;
      --i;
      continue;
    }
    int j = i - 4 > 0 ? i - 4 : 0;
    while (!bgv_exp_bit(e, j)) ++j;
    int w = 0;
    for (int q = i; q >= j; --q) w = (w << 1) | bgv_exp_bit(e, q);
    if (started) {
      s.step[s.n] = (uint32_t)(pending + (i - j + 1)) | ((uint32_t)(w >> 1) << 8);
      ++s.n;
    } else {
      s.first = w >> 1;
      started = true;
    }
    pending = 0;
    i = j - 1;
  }
  if (pending) {
    s.step[s.n] = (uint32_t)pending | (0xffu << 8);
    ++s.n;
  }
  return s;
}
#if defined(__HIPCC__)
#define BGV_CONSTANT __constant__
#else
#define BGV_CONSTANT
#endif
enum { BGV_POW_INV = 0, BGV_POW_P34 = 1, BGV_POW_SQRT = 2 };
static BGV_CONSTANT const bgv_pow_sched kBgvPow[3] = {
    bgv_make_sched(bgv_exp12{BGV_EXP_P_MINUS_2}, 381),
    bgv_make_sched(bgv_exp12{BGV_EXP_P_MINUS_3_DIV_4}, 379),
    bgv_make_sched(bgv_exp12{BGV_EXP_P_PLUS_1_DIV_4}, 379),
};

template <int W>
BGV_NOINLINE fp_t fp_pow_fixed(const fp_t& a) {
  const bgv_pow_sched& s = kBgvPow[W];
  fp_t tab[16];
  fp_t cur = a;
  tab[0] = a;
  const fp_t a2 = fp_sqr(a);
  BGV_NO_UNROLL for (int k = 1; k < 16; ++k) {
    cur = fp_mul(cur, a2);
    tab[k] = cur;
  }
  fp_t r = tab[s.first];
  BGV_NO_UNROLL for (int k = 0; k < s.n; ++k) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int ku = __builtin_amdgcn_readfirstlane(k);  // uniform: scalar loads of the schedule
#else
    const int ku = k;
#endif
    const uint32_t st = s.step[ku];
    const int d = (int)(st >> 8), nsq = (int)(st & 0xff);
    const fp_t m = tab[d & 15];
#if !defined(BGV_POW_CALLS)
    // the chain's products inline (one copy each in the loop): no call per squaring.  Round 6:
    // k_prep 12.46-12.48 vs 12.65-12.70 ms per 64,512-set launch, headline 2.655-2.663 vs
    // 2.636-2.640 M sets/s interleaved (profiles/r06/ab_powinl/); BGV_POW_CALLS keeps the calls
    BGV_NO_UNROLL for (int q = 0; q < nsq; ++q) {
      BGV_COUNT_SQR();
      r = fp_sqr_body(r);
    }
    if (d != 0xff) {
      BGV_COUNT_MUL();
      r = fp_mul_body(r, m);
    }
#else
    BGV_NO_UNROLL for (int q = 0; q < nsq; ++q) r = fp_sqr(r);
    if (d != 0xff) r = fp_mul(r, m);
#endif
  }
  return r;
}

BGV_HD fp_t fp_inv(const fp_t& a) { return fp_pow_fixed<BGV_POW_INV>(a); }

// a^((p-3)/4): for a QR, a * t = sqrt(a) and t = 1/sqrt(a).
BGV_HD fp_t fp_pow_p_minus_3_div_4(const fp_t& a) { return fp_pow_fixed<BGV_POW_P34>(a); }

// The fixed exponentiations of the square roots, as a policy: bgv_pow_lane runs them on the
// calling lane; bgv_wfp.h's bgv_pow_wave spreads each product over the wavefront (the latency
// path, one set per wave).  Same schedules, same values.
struct bgv_pow_lane {
  static BGV_HD fp_t p34(const fp_t& a) { return fp_pow_fixed<BGV_POW_P34>(a); }
  static BGV_HD fp_t sqrt_exp(const fp_t& a) { return fp_pow_fixed<BGV_POW_SQRT>(a); }
};

// sqrt candidate; returns true iff a is a square (then *out = a^((p+1)/4)).
template <class PW>
BGV_HD bool fp_sqrt_t(fp_t* out, const fp_t& a) {
  fp_t s = PW::sqrt_exp(a);
  *out = s;
  return fp_eq(fp_sqr(s), a);
}
BGV_HD bool fp_sqrt(fp_t* out, const fp_t& a) { return fp_sqrt_t<bgv_pow_lane>(out, a); }

// a / 2 mod p (a weakly reduced; the limb-0 parity is the value's parity)
BGV_HD fp_t fp_half(const fp_t& a) {
  const uint32_t m = 0u - (a.v[0] & 1);
  fp_t t;
  uint32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    uint32_t s = a.v[i] + (p_limb(i) & m) + c;
    t.v[i] = s & LMASK;
    c = s >> LBITS;
  }
  fp_t r;
  BGV_UNROLL for (int i = 0; i < NL - 1; ++i) r.v[i] = (t.v[i] >> 1) | ((t.v[i + 1] & 1) << (LBITS - 1));
  r.v[NL - 1] = t.v[NL - 1] >> 1;
  return r;  // (a + p) / 2 < 1.5p
}

// Compare canonical raw integers: a > b
BGV_HD bool fp_raw_gt(const fp_t& a, const fp_t& b) {
  int32_t c = 0;  // b - a borrows iff a > b
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)b.v[i] - (int32_t)a.v[i] + c;
    c = s >> LBITS;
  }
  return c < 0;
}

// raw integer < p ?
BGV_HD bool fp_raw_lt_p(const fp_t& a) {
  int32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)a.v[i] - (int32_t)p_limb(i) + c;
    c = s >> LBITS;
  }
  return c < 0;
}

// ZCash "lexicographically largest": raw(a) > (p-1)/2
BGV_HD bool fp_lex_largest(const fp_t& a_mont) {
  const fp_t half = {BGV_HALF_P_RAW};
  return fp_raw_gt(fp_from_mont(a_mont), half);
}

// bits [lo, lo+28) of a big-endian byte string of n bytes (bits past the top read 0)
BGV_HD uint32_t be_bits28(const uint8_t* b, int n, int lo) {
  uint32_t r = 0;
  BGV_UNROLL for (int k = 0; k < 5; ++k) {  // 28 bits touch at most 5 bytes
    const int bytepos = (lo >> 3) + k;     // byte index from the little end
    if (bytepos < n) r |= (uint32_t)((uint64_t)b[n - 1 - bytepos] << (8 * k) >> (lo & 7));
  }
  return r & LMASK;
}

// big-endian 48 bytes -> raw limbs
BGV_HD fp_t fp_from_be48(const uint8_t* b) {
  fp_t r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = be_bits28(b, 48, LBITS * i);
  return r;
}

// canonical raw limbs -> big-endian 48 bytes
BGV_HD void fp_to_be48(uint8_t* b, const fp_t& raw) {
  BGV_UNROLL for (int k = 0; k < 48; ++k) {
    const int bit = 8 * k;  // byte k from the little end
    const int li = bit / LBITS, sh = bit % LBITS;
    uint32_t v = raw.v[li] >> sh;
    if (sh > LBITS - 8 && li + 1 < NL) v |= raw.v[li + 1] << (LBITS - sh);
    b[47 - k] = (uint8_t)v;
  }
}

// ---------------------------------------------------------------------------
// Fp2
// ---------------------------------------------------------------------------
BGV_HD fp2_t fp2_zero() { return fp2_t{fp_zero(), fp_zero()}; }
BGV_HD fp2_t fp2_one() { return fp2_t{fp_one(), fp_zero()}; }
BGV_HD bool fp2_is_zero(const fp2_t& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
BGV_HD bool fp2_eq(const fp2_t& a, const fp2_t& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
BGV_HD fp2_t fp2_select(bool c, const fp2_t& a, const fp2_t& b) {
  return fp2_t{fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)};
}
BGV_HD fp2_t fp2_add(const fp2_t& a, const fp2_t& b) { return fp2_t{fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
BGV_HD fp2_t fp2_sub(const fp2_t& a, const fp2_t& b) { return fp2_t{fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
BGV_HD fp2_t fp2_dbl(const fp2_t& a) { return fp2_t{fp_dbl(a.c0), fp_dbl(a.c1)}; }
BGV_HD fp2_t fp2_neg(const fp2_t& a) { return fp2_t{fp_neg(a.c0), fp_neg(a.c1)}; }
BGV_HD fp2_t fp2_conj(const fp2_t& a) { return fp2_t{a.c0, fp_neg(a.c1)}; }

// Operand components: normalized limbs, values < 8p (fp6/fp12 Karatsuba sums made
// with fp2_add_norm); the operand sums below are then < 16p with limbs < 2^29,
// within fp_mul_l's bounds.  The result is weakly reduced.
#if defined(BGV_LZ2_WIDE)
// a unit with the deferred-reduction Fp2 products (bls_wide.h; defined in bls_lazy.h)
BGV_HD fp2_t fp2_mul_wide(const fp2_t& a, const fp2_t& b);
BGV_HD fp2_t fp2_sqr_wide(const fp2_t& a);
BGV_HD fp2_t fp2_mul_fp_wide(const fp2_t& a, const fp_t& s);
#endif
BGV_HD fp2_t fp2_mul(const fp2_t& a, const fp2_t& b) {
#if defined(BGV_LZ2_WIDE)
  return fp2_mul_wide(a, b);
#endif
  fp_t t0 = fp_mul(a.c0, b.c0);
  fp_t t1 = fp_mul(a.c1, b.c1);
  fp_t t2 = fp_mul(fp_add_nr(a.c0, a.c1), fp_add_nr(b.c0, b.c1));
  return fp2_t{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

// a weakly reduced (< 2p): (a0 + a1)(a0 - a1 + 2p) and (2 a0) a1, no reduced adds.
BGV_HD fp2_t fp2_sqr(const fp2_t& a) {
#if defined(BGV_LZ2_WIDE)
  return fp2_sqr_wide(a);
#endif
  return fp2_t{fp_mul(fp_add_nr(a.c0, a.c1), fp_sub_nr(a.c0, a.c1)), fp_mul(fp_add_nr(a.c0, a.c0), a.c1)};
}

// Karatsuba operand sum: normalized, unreduced (< 4p for reduced inputs)
BGV_HD fp2_t fp2_add_norm(const fp2_t& a, const fp2_t& b) {
  return fp2_t{fp_add_norm(a.c0, b.c0), fp_add_norm(a.c1, b.c1)};
}

BGV_HD fp2_t fp2_mul_fp(const fp2_t& a, const fp_t& b) {
#if defined(BGV_LZ2_WIDE)
  return fp2_mul_fp_wide(a, b);
#endif
  return fp2_t{fp_mul(a.c0, b), fp_mul(a.c1, b)};
}

// multiply by xi = 1 + i
BGV_HD fp2_t fp2_mul_xi(const fp2_t& a) { return fp2_t{fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

BGV_NOINLINE fp2_t fp2_inv(const fp2_t& a) {
  fp_t n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp_t ni = fp_inv(n);
  return fp2_t{fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}

BGV_HD fp2_t fp2_half(const fp2_t& a) { return fp2_t{fp_half(a.c0), fp_half(a.c1)}; }

// Square root in Fp2 (p = 3 mod 4) by the norm ("complex") method with one
// shared exponentiation for sqrt and inverse.  Returns false if a is not a
// square.  Any root is returned; callers fix the sign.
template <class PW>
BGV_NOINLINE bool fp2_sqrt_t(fp2_t* out, const fp2_t& a) {
  const fp_t n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp_t g;
  const bool n_sq = fp_sqrt_t<PW>(&g, n);
  const bool a1z = fp_is_zero(a.c1);
  // delta = a1 == 0 ? a0 : (a0 + g) / 2
  fp_t d = fp_select(a1z, fp_half(fp_add(a.c0, g)), a.c0);
  fp_t t = PW::p34(d);
  fp_t dt = fp_mul(d, t);
  fp_t s = fp_mul(dt, t);  // d^((p-1)/2)
  fp_t a1t2 = fp_half(fp_mul(a.c1, t));
  // s == 1: (d t, a1 t / 2);  s == -1: (a1 t / 2, -d t)
  const bool qr = fp_eq(s, fp_one());
  fp2_t y;
  y.c0 = fp_select(qr, a1t2, dt);
  y.c1 = fp_select(qr, fp_neg(dt), a1t2);
  *out = y;
  return n_sq && fp2_eq(fp2_sqr(y), a);
}
BGV_HD bool fp2_sqrt(fp2_t* out, const fp2_t& a) { return fp2_sqrt_t<bgv_pow_lane>(out, a); }

// RFC 9380 sgn0 for Fp2 (on raw values)
BGV_HD uint32_t fp2_sgn0(const fp2_t& a_mont) {
  fp_t a0 = fp_from_mont(a_mont.c0), a1 = fp_from_mont(a_mont.c1);
  uint32_t s0 = a0.v[0] & 1, s1 = a1.v[0] & 1;
  uint32_t z0 = fp_is_zero(a0) ? 1u : 0u;
  return s0 | (z0 & s1);
}

// ZCash sign for Fp2: c1 > (p-1)/2, or c1 == 0 and c0 > (p-1)/2
BGV_HD bool fp2_lex_largest(const fp2_t& a) {
  const bool c1z = fp_is_zero(a.c1);
  return c1z ? fp_lex_largest(a.c0) : fp_lex_largest(a.c1);
}

// ---------------------------------------------------------------------------
// Fp6
// ---------------------------------------------------------------------------
BGV_HD fp6_t fp6_zero() { return fp6_t{fp2_zero(), fp2_zero(), fp2_zero()}; }
BGV_HD fp6_t fp6_one() { return fp6_t{fp2_one(), fp2_zero(), fp2_zero()}; }
BGV_HD fp6_t fp6_add(const fp6_t& a, const fp6_t& b) {
  return fp6_t{fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)};
}
BGV_HD fp6_t fp6_sub(const fp6_t& a, const fp6_t& b) {
  return fp6_t{fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)};
}
BGV_HD fp6_t fp6_neg(const fp6_t& a) { return fp6_t{fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
BGV_HD fp6_t fp6_mul_v(const fp6_t& a) { return fp6_t{fp2_mul_xi(a.c2), a.c0, a.c1}; }

// Operand coefficients: normalized, values < 4p (an fp6_add_norm of reduced values
// at most); the result is weakly reduced.
BGV_MILLER_ATTR fp6_t fp6_mul(const fp6_t& a, const fp6_t& b) {
  fp2_t t0 = fp2_mul(a.c0, b.c0);
  fp2_t t1 = fp2_mul(a.c1, b.c1);
  fp2_t t2 = fp2_mul(a.c2, b.c2);
  fp2_t c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add_norm(a.c1, a.c2), fp2_add_norm(b.c1, b.c2)), t1), t2)),
                     t0);
  fp2_t c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add_norm(a.c0, a.c1), fp2_add_norm(b.c0, b.c1)), t0), t1),
                     fp2_mul_xi(t2));
  fp2_t c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add_norm(a.c0, a.c2), fp2_add_norm(b.c0, b.c2)), t0), t2), t1);
  return fp6_t{c0, c1, c2};
}

BGV_NOINLINE fp6_t fp6_sqr(const fp6_t& a) {
  // CH-SQR2
  fp2_t s0 = fp2_sqr(a.c0);
  fp2_t ab = fp2_mul(a.c0, a.c1);
  fp2_t s1 = fp2_dbl(ab);
  fp2_t s2 = fp2_sqr(fp2_add(fp2_sub(a.c0, a.c1), a.c2));
  fp2_t bc = fp2_mul(a.c1, a.c2);
  fp2_t s3 = fp2_dbl(bc);
  fp2_t s4 = fp2_sqr(a.c2);
  fp2_t c0 = fp2_add(fp2_mul_xi(s3), s0);
  fp2_t c1 = fp2_add(fp2_mul_xi(s4), s1);
  fp2_t c2 = fp2_sub(fp2_sub(fp2_add(fp2_add(s1, s2), s3), s0), s4);
  return fp6_t{c0, c1, c2};
}

// a * (b0 + b1 v)
BGV_MILLER_ATTR fp6_t fp6_mul_01(const fp6_t& a, const fp2_t& b0, const fp2_t& b1) {
  fp2_t t0 = fp2_mul(a.c0, b0);
  fp2_t t1 = fp2_mul(a.c1, b1);
  fp2_t c0 = fp2_add(fp2_mul_xi(fp2_mul(a.c2, b1)), t0);
  fp2_t c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add_norm(a.c0, a.c1), fp2_add_norm(b0, b1)), t0), t1);
  fp2_t c2 = fp2_add(fp2_mul(a.c2, b0), t1);
  return fp6_t{c0, c1, c2};
}

// a * (b1 v)
BGV_HD fp6_t fp6_mul_1(const fp6_t& a, const fp2_t& b1) {
  return fp6_t{fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

BGV_NOINLINE fp6_t fp6_inv(const fp6_t& a) {
  fp2_t t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2_t t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2_t t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2_t d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2_t di = fp2_inv(d);
  return fp6_t{fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di)};
}

// ---------------------------------------------------------------------------
// Fp12
// ---------------------------------------------------------------------------
BGV_HD fp12_t fp12_one() { return fp12_t{fp6_one(), fp6_zero()}; }

BGV_HD bool fp12_is_one(const fp12_t& a) {
  const fp12_t o = fp12_one();
  bool eq = true;
  const fp2_t* x = &a.c0.c0;
  const fp2_t* y = &o.c0.c0;
  BGV_UNROLL for (int i = 0; i < 6; ++i) eq = eq && fp2_eq(x[i], y[i]);
  return eq;
}

BGV_HD fp12_t fp12_conj(const fp12_t& a) { return fp12_t{a.c0, fp6_neg(a.c1)}; }

BGV_HD fp6_t fp6_add_norm(const fp6_t& a, const fp6_t& b) {
  return fp6_t{fp2_add_norm(a.c0, b.c0), fp2_add_norm(a.c1, b.c1), fp2_add_norm(a.c2, b.c2)};
}

BGV_NOINLINE fp12_t fp12_mul(const fp12_t& a, const fp12_t& b) {
  fp6_t t0 = fp6_mul(a.c0, b.c0);
  fp6_t t1 = fp6_mul(a.c1, b.c1);
  fp6_t c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add_norm(a.c0, a.c1), fp6_add_norm(b.c0, b.c1)), t0), t1);
  fp6_t c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12_t{c0, c1};
}

BGV_MILLER_ATTR fp12_t fp12_sqr(const fp12_t& a) {
  fp6_t t = fp6_mul(a.c0, a.c1);
  fp6_t s = fp6_mul(fp6_add_norm(a.c0, a.c1), fp6_add_norm(a.c0, fp6_mul_v(a.c1)));
  fp6_t c0 = fp6_sub(fp6_sub(s, t), fp6_mul_v(t));
  return fp12_t{c0, fp6_add(t, t)};
}

// f * (l0 + l1 w^2 + l3 w^3): a line with nonzero tower coefficients
// c0.c0 = l0, c0.c1 = l1, c1.c1 = l3.
BGV_MILLER_ATTR fp12_t fp12_mul_line(const fp12_t& f, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
  fp6_t t0 = fp6_mul_01(f.c0, l0, l1);
  fp6_t t1 = fp6_mul_1(f.c1, l3);
  fp6_t c1 = fp6_sub(fp6_sub(fp6_mul_01(fp6_add_norm(f.c0, f.c1), l0, fp2_add_norm(l1, l3)), t0), t1);
  fp6_t c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12_t{c0, c1};
}

BGV_NOINLINE fp12_t fp12_inv(const fp12_t& a) {
  fp6_t n = fp6_sub(fp6_sqr(a.c0), fp6_mul_v(fp6_sqr(a.c1)));
  fp6_t ni = fp6_inv(n);
  return fp12_t{fp6_mul(a.c0, ni), fp6_neg(fp6_mul(a.c1, ni))};
}

BGV_NOINLINE fp12_t fp12_frob(const fp12_t& a) {
  const fp2_t g[6] = BGV_FROB1;
  fp12_t r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), g[1]);
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), g[2]);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), g[3]);
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), g[4]);
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), g[5]);
  return r;
}

BGV_HD fp12_t fp12_frob2(const fp12_t& a) {
  const fp_t g[6] = BGV_FROB2;
  fp12_t r;
  r.c0.c0 = a.c0.c0;
  r.c0.c1 = fp2_mul_fp(a.c0.c1, g[1]);
  r.c0.c2 = fp2_mul_fp(a.c0.c2, g[2]);
  r.c1.c0 = fp2_mul_fp(a.c1.c0, g[3]);
  r.c1.c1 = fp2_mul_fp(a.c1.c1, g[4]);
  r.c1.c2 = fp2_mul_fp(a.c1.c2, g[5]);
  return r;
}

// Granger-Scott squaring, valid in the cyclotomic subgroup (after the easy part).
BGV_HD void fp4_sqr(fp2_t* c0, fp2_t* c1, const fp2_t& a, const fp2_t& b) {
  fp2_t t0 = fp2_sqr(a);
  fp2_t t1 = fp2_sqr(b);
  *c0 = fp2_add(fp2_mul_xi(t1), t0);
  *c1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(a, b)), t0), t1);
}

BGV_NOINLINE fp12_t fp12_cyclotomic_sqr(const fp12_t& f) {
  fp2_t z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2;
  fp2_t z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fp2_t t0, t1, t2, t3;
  fp4_sqr(&t0, &t1, z0, z1);
  z0 = fp2_sub(t0, z0);
  z0 = fp2_add(fp2_dbl(z0), t0);
  z1 = fp2_add(t1, z1);
  z1 = fp2_add(fp2_dbl(z1), t1);
  fp4_sqr(&t0, &t1, z2, z3);
  fp4_sqr(&t2, &t3, z4, z5);
  z4 = fp2_sub(t0, z4);
  z4 = fp2_add(fp2_dbl(z4), t0);
  z5 = fp2_add(t1, z5);
  z5 = fp2_add(fp2_dbl(z5), t1);
  t0 = fp2_mul_xi(t3);
  z2 = fp2_add(t0, z2);
  z2 = fp2_add(fp2_dbl(z2), t0);
  z3 = fp2_sub(t2, z3);
  z3 = fp2_add(fp2_dbl(z3), t2);
  return fp12_t{fp6_t{z0, z4, z3}, fp6_t{z2, z1, z5}};
}
