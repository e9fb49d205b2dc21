// Lazy Fp arithmetic with compile-time bounds (gfx950, one field element per lane).
//
// fp_t keeps every value normalized (limbs < 2^28) and weakly reduced (< 2p), so each
// fp_add / fp_sub is two 14-limb carry chains plus a conditional correction: ~100 VALU
// instructions, against ~490 for a whole Montgomery product.  The Miller loop and the
// G2 point formulas run ~3 such ops per product; the ISA of miller_loop1 had 35k inline
// instructions per doubling step beside 107 product calls (52k), mostly carry chains.
//
// lz<LM, VM> is an Fp value whose limbs are at most LM and whose value is below VM * p.
// Both bounds are template arguments, so every formula's intermediate bounds are derived
// by the compiler and every product checks its operands with a static_assert:
//   lz_add   limb-wise sum, 14 instructions          -> lz<LA + LB, VA + VB>
//   lz_sub   a + (k p - b) with a redundant representation of k p whose every limb
//            covers b's limb bound (built at compile time): 28 instructions, no borrow
//   lz_mul   fp_mul_l (28-bit row-wise Montgomery) takes any operands whose limb product
//            keeps its 64-bit column sums (14 rows of a_i b_j + m p_j, plus a carry)
//            below 2^64 and whose values keep ab/R + p below 2p (VA VB <= 2520 = R/p)
//   lz_norm  one carry chain (42 instructions): limbs < 2^28, value unchanged
//   lz_out   lz_norm, then minus q p with q from the top limb: an fp_t (< 2p) again
// The same source runs on the host (tests/hostsim), where -DBGV_LAZY_CHECK also checks
// every bound at run time.
#pragma once
#include "bls_field.h"

namespace lzc {
constexpr uint64_t P13 = 0x1a011;  // top limb of p
// largest limb product a_i * b_j fp_mul_l / fp_sqr_l accept: 14 (LA LB + 2^56) + 2^36 < 2^64
constexpr uint64_t MUL_LIMB_MAX = (~0ull - (1ull << 36)) / 14 - (1ull << 56);
constexpr uint64_t VMUL_MAX = 2520;  // floor(2^392 / p)
constexpr uint64_t cmax(uint64_t a, uint64_t b) { return a > b ? a : b; }

// k p in 14 limbs with limbs 0..12 >= lb and the top limb >= the top limb any value below
// vb p can have (or lb): the subtrahend's bounds.  k is the smallest that works.
struct kp {
  uint32_t v[NL];
  uint64_t maxl;
  uint64_t k;
};
constexpr kp make_kp(uint64_t lb, uint64_t vb) {
  const uint32_t P[NL] = BGV_P_LIMBS;
  const uint64_t topb = vb * (P13 + 1) < lb ? vb * (P13 + 1) : lb;
  kp out{};
  for (uint64_t k = 1; k < 4096; ++k) {
    int64_t L[NL] = {};
    uint64_t c = 0;
    for (int i = 0; i < NL; ++i) {
      const uint64_t t = k * P[i] + c;
      if (i < NL - 1) {
        L[i] = (int64_t)(t & LMASK);
        c = t >> LBITS;
      } else {
        L[i] = (int64_t)t;
      }
    }
    for (int i = 0; i < NL - 1; ++i) {
      if (L[i] < (int64_t)lb) {
        const int64_t d = ((int64_t)lb - L[i] + (int64_t)LMASK) >> LBITS;
        L[i] += d << LBITS;
        L[i + 1] -= d;
      }
    }
    if (L[NL - 1] < (int64_t)topb) continue;
    bool ok = true;
    uint64_t m = 0;
    for (int i = 0; i < NL; ++i) {
      if (L[i] < 0 || L[i] > 0xffffffffll) ok = false;
      m = cmax(m, (uint64_t)L[i]);
    }
    if (!ok) continue;
    for (int i = 0; i < NL; ++i) out.v[i] = (uint32_t)L[i];
    out.maxl = m;
    out.k = k;
    return out;
  }
  return out;  // k == 0: no representation (static_assert at the use)
}
}  // namespace lzc

#include "bls_wide.h"  // after lzc: its fixed k p come from make_kp

template <uint64_t LM, uint64_t VM>
struct lz {
  static_assert(LM <= 0xffffffffull, "lz: limb bound exceeds 32 bits");
  static_assert(VM >= 1 && VM <= 1000000, "lz: value bound out of range");
  static constexpr uint64_t L = LM, V = VM;
  uint32_t v[NL];
};

typedef lz<LMASK, 2> lzr;  // the fp_t invariant

#if defined(BGV_LAZY_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
#include <stdio.h>
#include <stdlib.h>
// value < vm * p and limbs <= lm, checked on the host build (out of line: one copy)
__attribute__((noinline)) static void lz_check_v(const uint32_t* v, uint64_t LM, uint64_t VM, const char* what) {
  const uint32_t P[NL] = BGV_P_LIMBS;
  for (int i = 0; i < NL; ++i)
    if (v[i] > LM) {
      fprintf(stderr, "lz bound: %s limb %d = %x > %llx\n", what, i, v[i], (unsigned long long)LM);
      abort();
    }
  // compare sum v_i 2^(28 i) with VM * p: normalize both into 28-bit digits
  unsigned __int128 ca = 0, cb = 0;
  int cmp = 0;
  uint32_t da[NL + 2], db[NL + 2];
  for (int i = 0; i < NL + 2; ++i) {
    if (i < NL) ca += v[i];
    if (i < NL) cb += (unsigned __int128)VM * P[i];
    da[i] = (uint32_t)(ca & LMASK);
    db[i] = (uint32_t)(cb & LMASK);
    ca >>= LBITS;
    cb >>= LBITS;
  }
  for (int i = NL + 1; i >= 0 && !cmp; --i) cmp = da[i] < db[i] ? -1 : (da[i] > db[i] ? 1 : 0);
  if (cmp >= 0) {
    fprintf(stderr, "lz bound: %s value >= %llu p\n", what, (unsigned long long)VM);
    abort();
  }
}
template <uint64_t LM, uint64_t VM>
inline void lz_check(const lz<LM, VM>& a, const char* what) {
  lz_check_v(a.v, LM, VM, what);
}
#define LZ_CHECK(x, w) lz_check(x, w)
#else
#define LZ_CHECK(x, w) ((void)0)
#endif

BGV_HD lzr lz_in(const fp_t& a) {
  lzr r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i];
  LZ_CHECK(r, "in");
  return r;
}

template <uint64_t L2, uint64_t V2, uint64_t LA, uint64_t VA>
BGV_HD lz<L2, V2> lz_widen(const lz<LA, VA>& a) {
  static_assert(LA <= L2 && VA <= V2, "lz_widen: narrowing");
  lz<L2, V2> r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i];
  return r;
}

template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD lz<LA + LB, VA + VB> lz_add(const lz<LA, VA>& a, const lz<LB, VB>& b) {
  lz<LA + LB, VA + VB> r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i] + b.v[i];
  LZ_CHECK(r, "add");
  return r;
}

template <uint64_t LA, uint64_t VA>
BGV_HD lz<2 * LA, 2 * VA> lz_dbl(const lz<LA, VA>& a) {
  return lz_add(a, a);
}

// a * M for a small constant M (shifts and shift-adds)
template <uint64_t M, uint64_t LA, uint64_t VA>
BGV_HD lz<LA * M, VA * M> lz_mulk(const lz<LA, VA>& a) {
  lz<LA * M, VA * M> r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i] * (uint32_t)M;
  LZ_CHECK(r, "mulk");
  return r;
}

template <uint64_t LB, uint64_t VB>
struct lz_sub_t {
  static constexpr lzc::kp K = lzc::make_kp(LB, VB);
  static_assert(K.k != 0, "lz_sub: no k p representation covers the subtrahend");
};

template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD lz<LA + lz_sub_t<LB, VB>::K.maxl, VA + lz_sub_t<LB, VB>::K.k> lz_sub(const lz<LA, VA>& a,
                                                                            const lz<LB, VB>& b) {
  constexpr lzc::kp K = lzc::make_kp(LB, VB);
  lz<LA + K.maxl, VA + K.k> r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i] + (K.v[i] - b.v[i]);
  LZ_CHECK(r, "sub");
  return r;
}

// k p - b: at most k p (b = 0), so the value bound is k + 1
template <uint64_t LB, uint64_t VB>
BGV_HD lz<lz_sub_t<LB, VB>::K.maxl, lz_sub_t<LB, VB>::K.k + 1> lz_neg(const lz<LB, VB>& b) {
  constexpr lzc::kp K = lzc::make_kp(LB, VB);
  lz<K.maxl, K.k + 1> r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = K.v[i] - b.v[i];
  LZ_CHECK(r, "neg");
  return r;
}

template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD lzr lz_mul(const lz<LA, VA>& a, const lz<LB, VB>& b) {
  static_assert(LA * LB <= lzc::MUL_LIMB_MAX, "lz_mul: limb product overflows the column sums");
  static_assert(VA * VB <= lzc::VMUL_MAX, "lz_mul: operand values too large for a < 2p result");
#if defined(BGV_LAZY_INLINE_MUL)
  BGV_COUNT_MUL();
  const fp_t r = fp_mul_body(fp_t{{BGV_V14(a)}}, fp_t{{BGV_V14(b)}});
#else
  const fp_t r = fp_mul_l(BGV_V14(a), BGV_V14(b));
#endif
  lzr o;
  BGV_UNROLL for (int i = 0; i < NL; ++i) o.v[i] = r.v[i];
  LZ_CHECK(o, "mul");
  return o;
}

template <uint64_t LA, uint64_t VA>
BGV_HD lzr lz_sqr(const lz<LA, VA>& a) {
  static_assert(LA < (1ull << 31), "lz_sqr: doubled limbs overflow 32 bits");
  static_assert(LA * LA <= lzc::MUL_LIMB_MAX, "lz_sqr: limb product overflows the column sums");
  static_assert(VA * VA <= lzc::VMUL_MAX, "lz_sqr: operand value too large for a < 2p result");
#if defined(BGV_LAZY_INLINE_MUL)
  BGV_COUNT_SQR();
  const fp_t r = fp_sqr_body(fp_t{{BGV_V14(a)}});
#else
  const fp_t r = fp_sqr_l(BGV_V14(a));
#endif
  lzr o;
  BGV_UNROLL for (int i = 0; i < NL; ++i) o.v[i] = r.v[i];
  LZ_CHECK(o, "sqr");
  return o;
}

// carry chain: limbs 0..12 < 2^28; the top limb is floor(value / 2^364) < VA (P13 + 1)
template <uint64_t LA, uint64_t VA>
BGV_HD lz<LMASK, VA> lz_norm(const lz<LA, VA>& a) {
  static_assert(VA * (lzc::P13 + 1) <= LMASK, "lz_norm: top limb would exceed 28 bits");
  static_assert(LA + (1ull << 5) <= 0xffffffffull, "lz_norm: carry overflow");
  lz<LMASK, VA> r;
  if constexpr (LA <= LMASK) {  // already normalized (a product, say): a copy
    BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i];
    return r;
  }
  uint32_t c = 0;
  BGV_UNROLL for (int i = 0; i < NL - 1; ++i) {
    const uint32_t s = a.v[i] + c;
    r.v[i] = s & LMASK;
    c = s >> LBITS;
  }
  r.v[NL - 1] = a.v[NL - 1] + c;
  LZ_CHECK(r, "norm");
  return r;
}

// back to the fp_t invariant in one signed carry chain: subtract q p with q = top / (P13 + 1)
// taken from the unnormalized top limb.  q p <= top 2^364 <= value (the lower limbs are
// non-negative), and value - q p < (P13 + 1 + q) 2^364 + sum_{i<13} a_i 2^(28 i)
// < p + (q + 1) 2^364 + 2^368 < 2p for any q < 2^16; the chain leaves limbs < 2^28.
template <uint64_t LA, uint64_t VA>
BGV_HD fp_t lz_out(const lz<LA, VA>& a) {
  fp_t r;
  if constexpr (LA <= LMASK && VA <= 2) {
    BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i];
  } else if constexpr (VA <= 2) {
    const lz<LMASK, VA> n = lz_norm(a);
    BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = n.v[i];
  } else {
    static_assert(LA / (lzc::P13 + 1) < (1ull << 16), "lz_out: quotient estimate too large");
    const uint32_t P_[NL] = BGV_P_LIMBS;
    const uint32_t q = a.v[NL - 1] / (uint32_t)(lzc::P13 + 1);
    int64_t c = 0;
    BGV_UNROLL for (int i = 0; i < NL - 1; ++i) {
      const int64_t s = (int64_t)a.v[i] - (int64_t)((uint64_t)q * P_[i]) + c;
      r.v[i] = (uint32_t)s & LMASK;
      c = s >> LBITS;
    }
    r.v[NL - 1] = (uint32_t)((int64_t)a.v[NL - 1] - (int64_t)((uint64_t)q * P_[NL - 1]) + c);
  }
  LZ_CHECK(lz_in(r), "out");
  return r;
}

template <uint64_t LA, uint64_t VA>
BGV_HD lzr lz_red(const lz<LA, VA>& a) {
  return lz_in(lz_out(a));
}

template <uint64_t LA, uint64_t VA>
BGV_HD lz<LA, VA> lz_sel(bool c, const lz<LA, VA>& a, const lz<LA, VA>& b) {
  lz<LA, VA> r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = c ? b.v[i] : a.v[i];
  return r;
}

template <uint64_t LA, uint64_t VA>
BGV_HD bool lz_is_zero(const lz<LA, VA>& a) {
  return fp_is_zero(lz_out(a));
}

// ---------------------------------------------------------------------------
// Fp2 (both coefficients share one bound pair)
// ---------------------------------------------------------------------------
template <uint64_t LM, uint64_t VM>
struct lz2 {
  lz<LM, VM> c0, c1;
};
typedef lz2<LMASK, 2> lz2r;

template <uint64_t L0, uint64_t V0, uint64_t L1, uint64_t V1>
BGV_HD lz2<lzc::cmax(L0, L1), lzc::cmax(V0, V1)> lz2_mk(const lz<L0, V0>& a, const lz<L1, V1>& b) {
  constexpr uint64_t L = lzc::cmax(L0, L1), V = lzc::cmax(V0, V1);
  return lz2<L, V>{lz_widen<L, V>(a), lz_widen<L, V>(b)};
}
BGV_HD lz2r lz2_in(const fp2_t& a) { return lz2r{lz_in(a.c0), lz_in(a.c1)}; }
template <uint64_t L2, uint64_t V2, uint64_t LA, uint64_t VA>
BGV_HD lz2<L2, V2> lz2_widen(const lz2<LA, VA>& a) {
  return lz2<L2, V2>{lz_widen<L2, V2>(a.c0), lz_widen<L2, V2>(a.c1)};
}
template <uint64_t LA, uint64_t VA>
BGV_HD fp2_t lz2_out(const lz2<LA, VA>& a) {
  return fp2_t{lz_out(a.c0), lz_out(a.c1)};
}
template <uint64_t LA, uint64_t VA>
BGV_HD lz2r lz2_red(const lz2<LA, VA>& a) {
  return lz2r{lz_red(a.c0), lz_red(a.c1)};
}
template <uint64_t LA, uint64_t VA>
BGV_HD lz2<LMASK, VA> lz2_norm(const lz2<LA, VA>& a) {
  return lz2<LMASK, VA>{lz_norm(a.c0), lz_norm(a.c1)};
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz2_add(const lz2<LA, VA>& a, const lz2<LB, VB>& b) {
  return lz2_mk(lz_add(a.c0, b.c0), lz_add(a.c1, b.c1));
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz2_sub(const lz2<LA, VA>& a, const lz2<LB, VB>& b) {
  return lz2_mk(lz_sub(a.c0, b.c0), lz_sub(a.c1, b.c1));
}
template <uint64_t LA, uint64_t VA>
BGV_HD auto lz2_dbl(const lz2<LA, VA>& a) {
  return lz2_mk(lz_dbl(a.c0), lz_dbl(a.c1));
}
template <uint64_t M, uint64_t LA, uint64_t VA>
BGV_HD auto lz2_mulk(const lz2<LA, VA>& a) {
  return lz2_mk(lz_mulk<M>(a.c0), lz_mulk<M>(a.c1));
}
template <uint64_t LA, uint64_t VA>
BGV_HD auto lz2_neg(const lz2<LA, VA>& a) {
  return lz2_mk(lz_neg(a.c0), lz_neg(a.c1));
}
template <uint64_t LA, uint64_t VA>
BGV_HD auto lz2_conj(const lz2<LA, VA>& a) {
  return lz2_mk(a.c0, lz_neg(a.c1));
}
// times xi = 1 + i
template <uint64_t LA, uint64_t VA>
BGV_HD auto lz2_mul_xi(const lz2<LA, VA>& a) {
  return lz2_mk(lz_sub(a.c0, a.c1), lz_add(a.c0, a.c1));
}
// Karatsuba: 3 products, the cross term as (a0 + a1)(b0 + b1) - (t0 + t1)
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz2_mul_c(const lz2<LA, VA>& a, const lz2<LB, VB>& b) {
  const lzr t0 = lz_mul(a.c0, b.c0);
  const lzr t1 = lz_mul(a.c1, b.c1);
  const lzr t2 = lz_mul(lz_add(a.c0, a.c1), lz_add(b.c0, b.c1));
  return lz2_mk(lz_norm(lz_sub(t0, t1)), lz_norm(lz_sub(t2, lz_add(t0, t1))));
}
// (a0 + a1)(a0 - a1), 2 a0 a1: two products, outputs < 2p normalized
template <uint64_t LA, uint64_t VA>
BGV_HD lz2r lz2_sqr_c(const lz2<LA, VA>& a) {
  return lz2r{lz_mul(lz_add(a.c0, a.c1), lz_sub(a.c0, a.c1)), lz_mul(lz_dbl(a.c0), a.c1)};
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD lz2r lz2_mul_fp_c(const lz2<LA, VA>& a, const lz<LB, VB>& s) {
  return lz2r{lz_mul(a.c0, s), lz_mul(a.c1, s)};
}

// The deferred-reduction forms (bls_wide.h): one out-of-line call per Fp2 operation, b (or s)
// through the lane's LDS slot.  Same field elements as the _c forms
// (tests/test_hostsim_math.py::test_wide_fp2_products_equal_classic).
template <uint64_t V>
BGV_HD lz2<LMASK, V> lz2_unpack(const bgv_u28& r) {
  lz2<LMASK, V> o;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    o.c0.v[i] = r[i];
    o.c1.v[i] = r[NL + i];
  }
  LZ_CHECK(o.c0, "wide re");
  LZ_CHECK(o.c1, "wide im");
  return o;
}
// b goes to the slot: its limbs must be within BGV_WMUL_LB and its values within BGV_WMUL_VB p
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz2_mul_w(const lz2<LA, VA>& a, const lz2<LB, VB>& b) {
  static_assert(bgvw::mul_ok(LA, LB), "lz2_mul_w: limb product overflows the column sums");
  constexpr uint64_t V = bgvw::mul_vout(VA, VB);
  static_assert(V != 0, "lz2_mul_w: operand values too large");
  uint32_t w[2 * NL];
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    w[i] = b.c0.v[i];
    w[NL + i] = b.c1.v[i];
  }
  wslot_put(w, 2 * NL);
  return lz2_unpack<V>(fp2_mul_w_l(BGV_V14(a.c0), BGV_V14(a.c1)));
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD lz2r lz2_mul_fp_w(const lz2<LA, VA>& a, const lz<LB, VB>& s) {
  static_assert(bgvw::mul2_ok(LA, LB), "lz2_mul_fp_w: limb product overflows the column sums");
  static_assert(VA * VB < lzc::VMUL_MAX, "lz2_mul_fp_w: operand values too large for a < 2p result");
  wslot_put(s.v, NL);
  return lz2_unpack<2>(fp2_mul_fp_w_l(BGV_V14(a.c0), BGV_V14(a.c1)));
}
template <uint64_t LA, uint64_t VA>
BGV_HD lz2r lz2_sqr_w(const lz2<LA, VA>& a) {
  static_assert(LA <= BGV_WSQR_LIMB && VA <= BGV_WSQR_V, "lz2_sqr_w: operand out of the squaring's bounds");
  return lz2_unpack<2>(fp2_sqr_w_l(BGV_V14(a.c0), BGV_V14(a.c1)));
}
// which operand of a product can take the slot (0: neither)
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
constexpr int lz2_wide_side() {
  if constexpr (bgvw::mul_ok(LA, LB) && bgvw::mul_vout(VA, VB) != 0) return 1;
  if constexpr (bgvw::mul_ok(LB, LA) && bgvw::mul_vout(VB, VA) != 0) return 2;
  return 0;
}

#if defined(BGV_LZ2_WIDE)
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz2_mul(const lz2<LA, VA>& a, const lz2<LB, VB>& b) {
  constexpr int side = lz2_wide_side<LA, VA, LB, VB>();
#if defined(BGV_LZ2_WIDE_STRICT)
  static_assert(side != 0, "lz2_mul: operands outside the deferred-reduction product's bounds");
#endif
  if constexpr (side == 1)
    return lz2_mul_w(a, b);
  else if constexpr (side == 2)
    return lz2_mul_w(b, a);
  else
    return lz2_mul_c(a, b);
}
template <uint64_t LA, uint64_t VA>
BGV_HD lz2r lz2_sqr(const lz2<LA, VA>& a) {
#if defined(BGV_LZ2_WIDE_STRICT)
  static_assert(LA <= BGV_WSQR_LIMB && VA <= BGV_WSQR_V, "lz2_sqr: operand outside the wide squaring's bounds");
#endif
  if constexpr (LA <= BGV_WSQR_LIMB && VA <= BGV_WSQR_V)
    return lz2_sqr_w(a);
  else
    return lz2_sqr_c(a);
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD lz2r lz2_mul_fp(const lz2<LA, VA>& a, const lz<LB, VB>& s) {
  if constexpr (bgvw::mul2_ok(LA, LB) && VA * VB < lzc::VMUL_MAX)
    return lz2_mul_fp_w(a, s);
  else
    return lz2_mul_fp_c(a, s);
}
#else
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz2_mul(const lz2<LA, VA>& a, const lz2<LB, VB>& b) {
  return lz2_mul_c(a, b);
}
template <uint64_t LA, uint64_t VA>
BGV_HD lz2r lz2_sqr(const lz2<LA, VA>& a) {
  return lz2_sqr_c(a);
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD lz2r lz2_mul_fp(const lz2<LA, VA>& a, const lz<LB, VB>& s) {
  return lz2_mul_fp_c(a, s);
}
#endif

// An operand normalized for the deferred-reduction product only (its limb bounds are tighter
// than the fully reduced product's): a no-op in the other units.
template <uint64_t LA, uint64_t VA>
BGV_HD auto lz2_wnorm(const lz2<LA, VA>& a) {
#if defined(BGV_LZ2_WIDE)
  return lz2_norm(a);
#else
  return a;
#endif
}

// The eager fp2_t products of bls_field.h in a BGV_LZ2_WIDE unit (declared there): operand
// components normalized (limbs < 2^28) with values < 8p, results weakly reduced (< 2p).
#if defined(BGV_LZ2_WIDE)
BGV_HD fp2_t fp2_from_w28(const bgv_u28& r) {
  fp2_t o;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    o.c0.v[i] = r[i];
    o.c1.v[i] = r[NL + i];
  }
  return o;
}
BGV_HD fp2_t fp2_mul_wide(const fp2_t& a, const fp2_t& b) {
  static_assert(bgvw::mul_ok(LMASK, LMASK) && bgvw::mul_vout(8, 8) == 2, "fp2_mul_wide: eager bounds");
  uint32_t w[2 * NL];
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    w[i] = b.c0.v[i];
    w[NL + i] = b.c1.v[i];
  }
  wslot_put(w, 2 * NL);
  return fp2_from_w28(fp2_mul_w_l(BGV_V14(a.c0), BGV_V14(a.c1)));
}
BGV_HD fp2_t fp2_sqr_wide(const fp2_t& a) {
  static_assert(LMASK <= BGV_WSQR_LIMB && 2 <= BGV_WSQR_V, "fp2_sqr_wide: eager bounds");
  return fp2_from_w28(fp2_sqr_w_l(BGV_V14(a.c0), BGV_V14(a.c1)));
}
BGV_HD fp2_t fp2_mul_fp_wide(const fp2_t& a, const fp_t& s) {
  static_assert(bgvw::mul2_ok(LMASK, LMASK) && 8 * 8 < lzc::VMUL_MAX, "fp2_mul_fp_wide: eager bounds");
  wslot_put(s.v, NL);
  return fp2_from_w28(fp2_mul_fp_w_l(BGV_V14(a.c0), BGV_V14(a.c1)));
}
#endif
template <uint64_t LA, uint64_t VA>
BGV_HD lz2<LA, VA> lz2_sel(bool c, const lz2<LA, VA>& a, const lz2<LA, VA>& b) {
  return lz2<LA, VA>{lz_sel(c, a.c0, b.c0), lz_sel(c, a.c1, b.c1)};
}

// ---------------------------------------------------------------------------
// Fp6 / Fp12 (one bound pair per value)
// ---------------------------------------------------------------------------
template <uint64_t LM, uint64_t VM>
struct lz6 {
  lz2<LM, VM> c0, c1, c2;
};
template <uint64_t LM, uint64_t VM>
struct lz12 {
  lz6<LM, VM> c0, c1;
};

template <uint64_t L0, uint64_t V0, uint64_t L1, uint64_t V1, uint64_t L2_, uint64_t V2_>
BGV_HD auto lz6_mk(const lz2<L0, V0>& a, const lz2<L1, V1>& b, const lz2<L2_, V2_>& c) {
  constexpr uint64_t L = lzc::cmax(lzc::cmax(L0, L1), L2_), V = lzc::cmax(lzc::cmax(V0, V1), V2_);
  return lz6<L, V>{lz2_widen<L, V>(a), lz2_widen<L, V>(b), lz2_widen<L, V>(c)};
}
template <uint64_t L2, uint64_t V2, uint64_t LA, uint64_t VA>
BGV_HD lz6<L2, V2> lz6_widen(const lz6<LA, VA>& a) {
  return lz6<L2, V2>{lz2_widen<L2, V2>(a.c0), lz2_widen<L2, V2>(a.c1), lz2_widen<L2, V2>(a.c2)};
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz6_add(const lz6<LA, VA>& a, const lz6<LB, VB>& b) {
  return lz6_mk(lz2_add(a.c0, b.c0), lz2_add(a.c1, b.c1), lz2_add(a.c2, b.c2));
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz6_sub(const lz6<LA, VA>& a, const lz6<LB, VB>& b) {
  return lz6_mk(lz2_sub(a.c0, b.c0), lz2_sub(a.c1, b.c1), lz2_sub(a.c2, b.c2));
}
template <uint64_t LA, uint64_t VA>
BGV_HD auto lz6_neg(const lz6<LA, VA>& a) {
  return lz6_mk(lz2_neg(a.c0), lz2_neg(a.c1), lz2_neg(a.c2));
}
template <uint64_t LA, uint64_t VA>
BGV_HD lz6<LMASK, VA> lz6_norm(const lz6<LA, VA>& a) {
  return lz6<LMASK, VA>{lz2_norm(a.c0), lz2_norm(a.c1), lz2_norm(a.c2)};
}
template <uint64_t LA, uint64_t VA>
BGV_HD lz6<LMASK, 2> lz6_red(const lz6<LA, VA>& a) {
  return lz6<LMASK, 2>{lz2_red(a.c0), lz2_red(a.c1), lz2_red(a.c2)};
}
// times v: (xi a2, a0, a1)
template <uint64_t LA, uint64_t VA>
BGV_HD auto lz6_mul_v(const lz6<LA, VA>& a) {
  return lz6_mk(lz2_mul_xi(a.c2), a.c0, a.c1);
}

// Karatsuba over Fp2 (6 Fp2 products); the sums are taken before the products and the
// differences after, all lazy
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
BGV_HD auto lz6_mul(const lz6<LA, VA>& a, const lz6<LB, VB>& b) {
  const auto t0 = lz2_mul(a.c0, b.c0);
  const auto t1 = lz2_mul(a.c1, b.c1);
  const auto t2 = lz2_mul(a.c2, b.c2);
  const auto c0 = lz2_add(lz2_mul_xi(lz2_sub(lz2_mul(lz2_add(a.c1, a.c2), lz2_add(b.c1, b.c2)), lz2_add(t1, t2))), t0);
  const auto c1 = lz2_add(lz2_sub(lz2_mul(lz2_add(a.c0, a.c1), lz2_add(b.c0, b.c1)), lz2_add(t0, t1)), lz2_mul_xi(t2));
  const auto c2 = lz2_add(lz2_sub(lz2_mul(lz2_add(a.c0, a.c2), lz2_add(b.c0, b.c2)), lz2_add(t0, t2)), t1);
  return lz6_norm(lz6_mk(c0, c1, c2));
}

// a * (b0 + b1 v)
template <uint64_t LA, uint64_t VA, uint64_t L0, uint64_t V0, uint64_t L1, uint64_t V1>
BGV_HD auto lz6_mul_01(const lz6<LA, VA>& a, const lz2<L0, V0>& b0, const lz2<L1, V1>& b1) {
  const auto t0 = lz2_mul(a.c0, b0);
  const auto t1 = lz2_mul(a.c1, b1);
  const auto c0 = lz2_add(lz2_mul_xi(lz2_mul(a.c2, b1)), t0);
  const auto c1 = lz2_sub(lz2_mul(lz2_add(a.c0, a.c1), lz2_add(b0, b1)), lz2_add(t0, t1));
  const auto c2 = lz2_add(lz2_mul(a.c2, b0), t1);
  return lz6_norm(lz6_mk(c0, c1, c2));
}

// a * (b1 v)
template <uint64_t LA, uint64_t VA, uint64_t L1, uint64_t V1>
BGV_HD auto lz6_mul_1(const lz6<LA, VA>& a, const lz2<L1, V1>& b1) {
  return lz6_norm(lz6_mk(lz2_mul_xi(lz2_mul(a.c2, b1)), lz2_mul(a.c0, b1), lz2_mul(a.c1, b1)));
}

template <uint64_t LA, uint64_t VA>
BGV_HD lz12<LMASK, VA> lz12_norm(const lz12<LA, VA>& a) {
  return lz12<LMASK, VA>{lz6_norm(a.c0), lz6_norm(a.c1)};
}
template <uint64_t LA, uint64_t VA>
BGV_HD lz12<LMASK, 2> lz12_red(const lz12<LA, VA>& a) {
  return lz12<LMASK, 2>{lz6_red(a.c0), lz6_red(a.c1)};
}

BGV_HD lz12<LMASK, 2> lz12_in(const fp12_t& a) {
  return lz12<LMASK, 2>{lz6<LMASK, 2>{lz2_in(a.c0.c0), lz2_in(a.c0.c1), lz2_in(a.c0.c2)},
                        lz6<LMASK, 2>{lz2_in(a.c1.c0), lz2_in(a.c1.c1), lz2_in(a.c1.c2)}};
}
template <uint64_t LA, uint64_t VA>
BGV_HD fp12_t lz12_out(const lz12<LA, VA>& a) {
  return fp12_t{fp6_t{lz2_out(a.c0.c0), lz2_out(a.c0.c1), lz2_out(a.c0.c2)},
                fp6_t{lz2_out(a.c1.c0), lz2_out(a.c1.c1), lz2_out(a.c1.c2)}};
}

// (a0 + a1 w)^2 = (a0 + a1)(a0 + v a1) - t - v t + 2t w, t = a0 a1
template <uint64_t LA, uint64_t VA>
BGV_HD auto lz12_sqr(const lz12<LA, VA>& a) {
  const auto t = lz6_mul(a.c0, a.c1);
  const auto s = lz6_mul(lz6_norm(lz6_add(a.c0, a.c1)), lz6_norm(lz6_add(a.c0, lz6_mul_v(a.c1))));
  const auto c0 = lz6_sub(s, lz6_add(t, lz6_mul_v(t)));
  return lz12<lzc::cmax(decltype(c0.c0.c0)::L, 2 * decltype(t.c0.c0)::L),
              lzc::cmax(decltype(c0.c0.c0)::V, 2 * decltype(t.c0.c0)::V)>{
      lz6_widen<lzc::cmax(decltype(c0.c0.c0)::L, 2 * decltype(t.c0.c0)::L),
                lzc::cmax(decltype(c0.c0.c0)::V, 2 * decltype(t.c0.c0)::V)>(c0),
      lz6_widen<lzc::cmax(decltype(c0.c0.c0)::L, 2 * decltype(t.c0.c0)::L),
                lzc::cmax(decltype(c0.c0.c0)::V, 2 * decltype(t.c0.c0)::V)>(lz6_add(t, t))};
}

// f * (l0 + l1 w^2 + l3 w^3): tower coefficients c0.c0 = l0, c0.c1 = l1, c1.c1 = l3
template <uint64_t LA, uint64_t VA, uint64_t L0, uint64_t V0, uint64_t L1, uint64_t V1, uint64_t L3, uint64_t V3>
BGV_HD auto lz12_mul_line(const lz12<LA, VA>& f, const lz2<L0, V0>& l0, const lz2<L1, V1>& l1,
                          const lz2<L3, V3>& l3) {
  const auto t0 = lz6_mul_01(f.c0, l0, l1);
  const auto t1 = lz6_mul_1(f.c1, l3);
  const auto c1 = lz6_sub(lz6_mul_01(lz6_norm(lz6_add(f.c0, f.c1)), l0, lz2_norm(lz2_add(l1, l3))), lz6_add(t0, t1));
  const auto c0 = lz6_add(t0, lz6_mul_v(t1));
  constexpr uint64_t L = lzc::cmax(decltype(c0.c0.c0)::L, decltype(c1.c0.c0)::L);
  constexpr uint64_t V = lzc::cmax(decltype(c0.c0.c0)::V, decltype(c1.c0.c0)::V);
  return lz12<L, V>{lz6_widen<L, V>(c0), lz6_widen<L, V>(c1)};
}

// ---------------------------------------------------------------------------
// One name set over lz (Fp) and lz2 (Fp2), so the point formulas (bls_curve.h) are
// written once for G1 and G2.
// ---------------------------------------------------------------------------
BGV_HD lzr L_in(const fp_t& a) { return lz_in(a); }
BGV_HD lz2r L_in(const fp2_t& a) { return lz2_in(a); }
template <uint64_t A, uint64_t B> BGV_HD fp_t L_out(const lz<A, B>& a) { return lz_out(a); }
template <uint64_t A, uint64_t B> BGV_HD fp2_t L_out(const lz2<A, B>& a) { return lz2_out(a); }
template <uint64_t A, uint64_t B> BGV_HD lzr L_red(const lz<A, B>& a) { return lz_red(a); }
template <uint64_t A, uint64_t B> BGV_HD lz2r L_red(const lz2<A, B>& a) { return lz2_red(a); }
template <uint64_t A, uint64_t B> BGV_HD auto L_norm(const lz<A, B>& a) { return lz_norm(a); }
template <uint64_t A, uint64_t B> BGV_HD auto L_norm(const lz2<A, B>& a) { return lz2_norm(a); }
// an operand of a product normalized where the deferred-reduction Fp2 product needs it
template <uint64_t A, uint64_t B> BGV_HD auto L_wnorm(const lz<A, B>& a) { return a; }
template <uint64_t A, uint64_t B> BGV_HD auto L_wnorm(const lz2<A, B>& a) { return lz2_wnorm(a); }
template <uint64_t A, uint64_t B, uint64_t C, uint64_t D>
BGV_HD auto L_add(const lz<A, B>& a, const lz<C, D>& b) { return lz_add(a, b); }
template <uint64_t A, uint64_t B, uint64_t C, uint64_t D>
BGV_HD auto L_add(const lz2<A, B>& a, const lz2<C, D>& b) { return lz2_add(a, b); }
template <uint64_t A, uint64_t B, uint64_t C, uint64_t D>
BGV_HD auto L_sub(const lz<A, B>& a, const lz<C, D>& b) { return lz_sub(a, b); }
template <uint64_t A, uint64_t B, uint64_t C, uint64_t D>
BGV_HD auto L_sub(const lz2<A, B>& a, const lz2<C, D>& b) { return lz2_sub(a, b); }
template <uint64_t A, uint64_t B> BGV_HD auto L_dbl(const lz<A, B>& a) { return lz_dbl(a); }
template <uint64_t A, uint64_t B> BGV_HD auto L_dbl(const lz2<A, B>& a) { return lz2_dbl(a); }
template <uint64_t M, uint64_t A, uint64_t B> BGV_HD auto L_mulk(const lz<A, B>& a) { return lz_mulk<M>(a); }
template <uint64_t M, uint64_t A, uint64_t B> BGV_HD auto L_mulk(const lz2<A, B>& a) { return lz2_mulk<M>(a); }
template <uint64_t A, uint64_t B, uint64_t C, uint64_t D>
BGV_HD lzr L_mul(const lz<A, B>& a, const lz<C, D>& b) { return lz_mul(a, b); }
template <uint64_t A, uint64_t B, uint64_t C, uint64_t D>
BGV_HD auto L_mul(const lz2<A, B>& a, const lz2<C, D>& b) { return lz2_mul(a, b); }
template <uint64_t A, uint64_t B> BGV_HD lzr L_sqr(const lz<A, B>& a) { return lz_sqr(a); }
template <uint64_t A, uint64_t B> BGV_HD lz2r L_sqr(const lz2<A, B>& a) { return lz2_sqr(a); }
template <uint64_t A, uint64_t B> BGV_HD bool L_is_zero(const lz<A, B>& a) { return fp_is_zero(lz_out(a)); }
template <uint64_t A, uint64_t B> BGV_HD bool L_is_zero(const lz2<A, B>& a) { return fp2_is_zero(lz2_out(a)); }
