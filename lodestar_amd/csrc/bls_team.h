// Team-parallel Fp12 arithmetic for the group closing (final exponentiation).
//
// The per-set kernels keep one signature set per lane: thousands of independent
// chains fill the chip.  A group closing is different: one final exponentiation
// per device group, a few thousand groups per launch, each a serial chain of
// ~340 Fp12 squarings/products.  Run one lane per group and the closing is
// latency-bound (one wave per SIMD, a third of the SIMDs busy).  Here a TEAM of
// 16 lanes owns one Fp12 value: lane c < 12 holds one Fp coefficient in the
// w-basis,
//
//     f = sum_{k<6} f_k w^k,  w^6 = xi = 1 + u,  f_k = re + im u,  c = 2k + (re ? 0 : 1)
//
// (tower position of w^k: k even -> c0.c[k/2], k odd -> c1.c[k/2]), and a product
// is computed coefficient-parallel: lane (k, e) accumulates the 12 double-width
// Fp products that make up its coefficient (negations folded into operands as
// 2p - x, so every term is positive) and does ONE Montgomery reduction.  Operands
// are exchanged through LDS.  Per lane that is 12 x 196 + 196 u32 MACs against
// 54 full Fp products (~21k MACs) for the one-lane tower product.
//
// Final exponentiation without an inversion.  f^((p^12-1)/r) == 1 iff
// f^((p^2+1) h) lies in Fp6 (the kernel of x -> x^(p^6-1)), h = (p^4-p^2+1)/r.
// Modulo Fp6*, conj(a) = a^(p^6) = N(a)/a is an inverse of a for EVERY a, and the
// Frobenius maps are automorphisms, so the x-chain of the hard part
// (bls_pairing.h final_exp) runs unchanged on representatives with generic
// squarings, starting from t = frob2(f) * f; the verdict is "odd w-coefficients of
// the result are zero".  The easy part's Fp12 inversion disappears.
#pragma once
#include "bls_pairing.h"

#define BGV_TEAM 16
#define BGV_TEAM_COMPS 12

// fp_t index inside fp12_t of w-basis component c
BGV_HD int tm_fp_index(int c) {
  const int k = c >> 1, e = c & 1;
  return 2 * ((k & 1) * 3 + (k >> 1)) + e;
}

// t += x * y over 2 NL columns.  With limbs < 2^28 each column takes < 2^56 per
// term and 14 terms per product: 12 products stay below 2^63.4.
BGV_HD void wide_mac(uint64_t* t, const fp_t& x, const fp_t& y) {
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    BGV_UNROLL for (int j = 0; j < NL; ++j) t[i + j] += (uint64_t)x.v[i] * y.v[j];
  }
}

// Montgomery reduction of a double-width column sum T < 96 p^2 -> T / 2^392 mod p,
// result < 1.07 p (weakly reduced).  Same rows as fp_sqr_l's reduction.
BGV_HD fp_t wide_redc(uint64_t* t) {
  const uint32_t P_[NL] = BGV_P_LIMBS;
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

// Coefficient c = 2k + e of a * b (A, B: the 12 w-basis components of each factor).
//   c_k = sum_{i+j=k} a_i b_j + xi sum_{i+j=k+6} a_i b_j,  xi (y0 + y1 u) = (y0 - y1) + (y0 + y1) u
// re(a_i b_j) = x0 y0 + (-x1) y1        im(a_i b_j) = x0 y1 + x1 y0
// re(xi a_i b_j) = x0 (y0 - y1) + (-x1)(y0 + y1)    im(xi a_i b_j) = x0 (y0 + y1) + x1 (y0 - y1)
BGV_HD fp_t tm_mul_lane(int c, const fp_t* A, const fp_t* B) {
  const int k = c >> 1, e = c & 1;
  uint64_t t[2 * NL];
  BGV_UNROLL for (int q = 0; q < 2 * NL; ++q) t[q] = 0;
  BGV_NO_UNROLL for (int i = 0; i < 6; ++i) {
    const bool wrap = i > k;
    const int j = wrap ? k + 6 - i : k - i;
    const fp_t x0 = A[2 * i], x1 = A[2 * i + 1];
    const fp_t y0 = B[2 * j], y1 = B[2 * j + 1];
    const fp_t d = fp_sub_nr(y0, y1);    // y0 - y1 + 2p in (0, 4p)
    const fp_t s = fp_add_norm(y0, y1);  // < 4p
    const fp_t x1n = fp_sub_nr(fp_zero(), x1);  // 2p - x1 in (0, 2p]
    const fp_t X2 = fp_select(e != 0, x1n, x1);
    const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y0, y1);
    const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y1, y0);
    wide_mac(t, x0, Y1);
    wide_mac(t, X2, Y2);
  }
  return wide_redc(t);
}

// Coefficient c = 2k + e of a^2 with 7 double-width products instead of 12.  The
// ordered pairs (i, j) and (j, i) of c_k = sum_{i+j = k (mod 6)} a_i a_j (xi-scaled when
// i + j >= 6) carry the same product, so every lane takes 3 unordered pairs with the
// generic two-product formula of tm_mul_lane, the x operand doubled for a cross pair
// (i != j), plus, for even k, the unwrapped diagonal a_{k/2}^2 as one product:
// re = (x0 + x1)(x0 - x1), im = (2 x0) x1.  Pairs per k (i, j, wrap):
//   k=0: (1,5,w) (2,4,w) (3,3,w) + diag 0     k=1: (0,1) (2,5,w) (3,4,w)
//   k=2: (0,2) (3,5,w) (4,4,w) + diag 1       k=3: (0,3) (1,2) (4,5,w)
//   k=4: (0,4) (1,3) (5,5,w) + diag 2         k=5: (0,5) (1,4) (2,3)
// Every lane runs the same 7 products (odd k multiplies zeros in the 7th), so a team
// never diverges.  Bounds: operands < 4p, 7 products < 112 p^2, columns < 2^63.
BGV_HD fp_t tm_sqr_lane(int c, const fp_t* A) {
  const int k = c >> 1, e = c & 1;
  // packed (i, j, wrap) per pair slot, indexed by k
  const uint32_t kI[6] = {0x321, 0x320, 0x430, 0x410, 0x510, 0x210};
  const uint32_t kJ[6] = {0x345, 0x451, 0x452, 0x523, 0x534, 0x345};
  const uint32_t kW[6] = {0x7, 0x6, 0x6, 0x4, 0x4, 0x0};
  uint64_t t[2 * NL];
  BGV_UNROLL for (int q = 0; q < 2 * NL; ++q) t[q] = 0;
  BGV_NO_UNROLL for (int p = 0; p < 3; ++p) {
    const int i = (kI[k] >> (4 * p)) & 0xf, j = (kJ[k] >> (4 * p)) & 0xf;
    const bool wrap = (kW[k] >> p) & 1;
    const fp_t x0 = A[2 * i], x1 = A[2 * i + 1];
    const fp_t y0 = A[2 * j], y1 = A[2 * j + 1];
    const fp_t d = fp_sub_nr(y0, y1);
    const fp_t s = fp_add_norm(y0, y1);
    const fp_t x1n = fp_sub_nr(fp_zero(), x1);
    const fp_t X2n = fp_select(e != 0, x1n, x1);
    const bool cross = i != j;  // a cross pair is counted twice
    const fp_t X1 = fp_select(cross, x0, fp_add_norm(x0, x0));
    const fp_t X2 = fp_select(cross, X2n, fp_add_norm(X2n, X2n));
    const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y0, y1);
    const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y1, y0);
    wide_mac(t, X1, Y1);
    wide_mac(t, X2, Y2);
  }
  // unwrapped diagonal (even k): re (x0 + x1)(x0 - x1 + 2p), im (2 x0) x1; odd k adds 0
  const int h = k >> 1;
  const fp_t x0 = A[2 * h], x1 = A[2 * h + 1];
  const bool even = (k & 1) == 0;
  const fp_t P = e ? fp_add_norm(x0, x0) : fp_add_norm(x0, x1);
  const fp_t Q = e ? x1 : fp_sub_nr(x0, x1);
  wide_mac(t, fp_select(even, fp_zero(), P), Q);
  return wide_redc(t);
}

// Wide products (the latency path's final exponentiation): coefficient c is split over four
// lanes q = 0..3, each accumulating part of its double-width products and reducing them
// (REDC is linear, so the four results sum to the coefficient mod p).  A product then costs a
// lane 4 double-width products + 1 reduction instead of 12 + 1, a squaring 2 + 1 instead of
// 7 + 1.  Parts of tm_mul_lane's six i-terms: q0 {0, 4}, q1 {1, 5}, q2 {2}, q3 {3}; of
// tm_sqr_lane's three pairs and the diagonal: one each.  Each part is < 2p (few products).
BGV_HD fp_t tm_mul_part(int c, int q, const fp_t* A, const fp_t* B) {
  const int k = c >> 1, e = c & 1;
  uint64_t t[2 * NL];
  BGV_UNROLL for (int z = 0; z < 2 * NL; ++z) t[z] = 0;
  BGV_UNROLL for (int r = 0; r < 2; ++r) {
    const int i = q + 4 * r;
    const bool live = i < 6;
    const int ii = live ? i : 0;
    const bool wrap = ii > k;
    const int j = wrap ? k + 6 - ii : k - ii;
    const fp_t x0 = A[2 * ii], x1 = A[2 * ii + 1];
    const fp_t y0 = B[2 * j], y1 = B[2 * j + 1];
    const fp_t d = fp_sub_nr(y0, y1);
    const fp_t s = fp_add_norm(y0, y1);
    const fp_t x1n = fp_sub_nr(fp_zero(), x1);
    const fp_t X2 = fp_select(e != 0, x1n, x1);
    const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y0, y1);
    const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y1, y0);
    const fp_t z = fp_zero();
    wide_mac(t, live ? x0 : z, Y1);  // the second term of q2 / q3 multiplies zeros
    wide_mac(t, live ? X2 : z, Y2);
  }
  return wide_redc(t);
}

BGV_HD fp_t tm_sqr_part(int c, int q, const fp_t* A) {
  const int k = c >> 1, e = c & 1;
  const uint32_t kI[6] = {0x321, 0x320, 0x430, 0x410, 0x510, 0x210};
  const uint32_t kJ[6] = {0x345, 0x451, 0x452, 0x523, 0x534, 0x345};
  const uint32_t kW[6] = {0x7, 0x6, 0x6, 0x4, 0x4, 0x0};
  uint64_t t[2 * NL];
  BGV_UNROLL for (int z = 0; z < 2 * NL; ++z) t[z] = 0;
  const int p = q < 3 ? q : 0;
  const int i = (kI[k] >> (4 * p)) & 0xf, j = (kJ[k] >> (4 * p)) & 0xf;
  const bool wrap = (kW[k] >> p) & 1;
  const fp_t x0 = A[2 * i], x1 = A[2 * i + 1];
  const fp_t y0 = A[2 * j], y1 = A[2 * j + 1];
  const fp_t d = fp_sub_nr(y0, y1);
  const fp_t s = fp_add_norm(y0, y1);
  const fp_t x1n = fp_sub_nr(fp_zero(), x1);
  const fp_t X2n = fp_select(e != 0, x1n, x1);
  const bool cross = i != j;
  const fp_t X1 = fp_select(cross, x0, fp_add_norm(x0, x0));
  const fp_t X2 = fp_select(cross, X2n, fp_add_norm(X2n, X2n));
  const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y0, y1);
  const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y1, y0);
  // q3: the unwrapped diagonal (even k) as in tm_sqr_lane, zero for odd k
  const int h = k >> 1;
  const fp_t h0 = A[2 * h], h1 = A[2 * h + 1];
  const bool diag = q == 3, even = (k & 1) == 0;
  const fp_t P = e ? fp_add_norm(h0, h0) : fp_add_norm(h0, h1);
  const fp_t Q = e ? h1 : fp_sub_nr(h0, h1);
  const fp_t z = fp_zero();
  wide_mac(t, diag ? (even ? P : z) : X1, diag ? Q : Y1);
  wide_mac(t, diag ? z : X2, Y2);
  return wide_redc(t);
}

// tm_mul_line_lane split the same way: the three line terms on parts 0..2, part 3 adds 0
BGV_HD fp_t tm_mul_line_part(int c, int q, const fp_t* A, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
  const int k = c >> 1, e = c & 1;
  uint64_t t[2 * NL];
  BGV_UNROLL for (int z = 0; z < 2 * NL; ++z) t[z] = 0;
  const int term = q < 3 ? q : 0;
  const int j = term == 0 ? 0 : term + 1;  // 0, 2, 3
  const fp2_t& y = term == 0 ? l0 : (term == 1 ? l1 : l3);
  const bool wrap = k < j;
  const int i = wrap ? k - j + 6 : k - j;
  const fp_t x0 = A[2 * i], x1 = A[2 * i + 1];
  const fp_t d = fp_sub_nr(y.c0, y.c1);
  const fp_t s = fp_add_norm(y.c0, y.c1);
  const fp_t x1n = fp_sub_nr(fp_zero(), x1);
  const fp_t X2 = fp_select(e != 0, x1n, x1);
  const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y.c0, y.c1);
  const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y.c1, y.c0);
  const fp_t z = fp_zero();
  wide_mac(t, q < 3 ? x0 : z, Y1);
  wide_mac(t, q < 3 ? X2 : z, Y2);
  return wide_redc(t);
}

// Eight-part forms for a block of >= 96 lanes (k_final_fold): every double-width product of
// a coefficient on a lane of its own where the four-part forms pair them up.  mul: part q < 6
// the two products of a_q b_j (q = 6, 7 multiply zeros); sqr: parts 2p, 2p + 1 the two
// products of pair p of tm_sqr_part, part 6 the diagonal, part 7 zeros; mul_line: parts 2t,
// 2t + 1 the two products of line term t.  Same products as the four-part forms, regrouped.
BGV_HD fp_t tm_mul_part8(int c, int q, const fp_t* A, const fp_t* B) {
  const int k = c >> 1, e = c & 1;
  uint64_t t[2 * NL];
  BGV_UNROLL for (int z = 0; z < 2 * NL; ++z) t[z] = 0;
  const bool live = q < 6;
  const int i = live ? q : 0;
  const bool wrap = i > k;
  const int j = wrap ? k + 6 - i : k - i;
  const fp_t x0 = A[2 * i], x1 = A[2 * i + 1];
  const fp_t y0 = B[2 * j], y1 = B[2 * j + 1];
  const fp_t d = fp_sub_nr(y0, y1);
  const fp_t s = fp_add_norm(y0, y1);
  const fp_t x1n = fp_sub_nr(fp_zero(), x1);
  const fp_t X2 = fp_select(e != 0, x1n, x1);
  const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y0, y1);
  const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y1, y0);
  const fp_t z = fp_zero();
  wide_mac(t, live ? x0 : z, Y1);
  wide_mac(t, live ? X2 : z, Y2);
  return wide_redc(t);
}

BGV_HD fp_t tm_sqr_part8(int c, int q, const fp_t* A) {
  const int k = c >> 1, e = c & 1;
  const uint32_t kI[6] = {0x321, 0x320, 0x430, 0x410, 0x510, 0x210};
  const uint32_t kJ[6] = {0x345, 0x451, 0x452, 0x523, 0x534, 0x345};
  const uint32_t kW[6] = {0x7, 0x6, 0x6, 0x4, 0x4, 0x0};
  uint64_t t[2 * NL];
  BGV_UNROLL for (int z = 0; z < 2 * NL; ++z) t[z] = 0;
  const int p = q < 6 ? q >> 1 : 0;
  const int i = (kI[k] >> (4 * p)) & 0xf, j = (kJ[k] >> (4 * p)) & 0xf;
  const bool wrap = (kW[k] >> p) & 1;
  const fp_t x0 = A[2 * i], x1 = A[2 * i + 1];
  const fp_t y0 = A[2 * j], y1 = A[2 * j + 1];
  const fp_t d = fp_sub_nr(y0, y1);
  const fp_t s = fp_add_norm(y0, y1);
  const fp_t x1n = fp_sub_nr(fp_zero(), x1);
  const fp_t X2n = fp_select(e != 0, x1n, x1);
  const bool cross = i != j;
  const fp_t X1 = fp_select(cross, x0, fp_add_norm(x0, x0));
  const fp_t X2 = fp_select(cross, X2n, fp_add_norm(X2n, X2n));
  const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y0, y1);
  const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y1, y0);
  const int h = k >> 1;
  const fp_t h0 = A[2 * h], h1 = A[2 * h + 1];
  const bool even = (k & 1) == 0;
  const fp_t Pd = e ? fp_add_norm(h0, h0) : fp_add_norm(h0, h1);
  const fp_t Qd = e ? h1 : fp_sub_nr(h0, h1);
  const fp_t z = fp_zero();
  const fp_t X = q < 6 ? ((q & 1) ? X2 : X1) : (q == 6 && even ? Pd : z);
  const fp_t Y = q < 6 ? ((q & 1) ? Y2 : Y1) : Qd;
  wide_mac(t, X, Y);
  return wide_redc(t);
}

// Lean operands for the eight-part squaring.  A lane of k_final_fold keeps its (c, q) for the
// whole final exponentiation, and tm_sqr_part8 needs ONE X and ONE Y of the many it computes
// and selects between (d, s, 2p - x1, doubled forms, the diagonal's sums).  Each is an exact
// integer u1 S[i1] + u2 S[i2] + k p (|u| <= 2, k p keeping it >= 0), so a lane can evaluate
// just its own from a recipe fixed at kernel start: one 14-limb signed chain per operand.
// The integers are those tm_sqr_part8 forms, carry-normalized the same way, so the products
// and parts are bit-identical (tests/test_hostsim_math.py).
struct tm_lin_t {
  int i1, i2, u1, u2, k;
};

// Components have limbs < 2^28 below the top one and values < 2p: every limb sum
// u1 a + u2 b + k p_l + carry stays within 2^31, so the chain runs in 32-bit signed arithmetic.
BGV_HD fp_t tm_lin(const fp_t* S, const tm_lin_t& r) {
  const fp_t a = S[r.i1], b = S[r.i2];
  const uint32_t P_[NL] = BGV_P_LIMBS;
  fp_t o;
  int32_t cy = 0;
  BGV_UNROLL for (int l = 0; l < NL - 1; ++l) {
    const int32_t s = r.u1 * (int32_t)a.v[l] + r.u2 * (int32_t)b.v[l] + r.k * (int32_t)P_[l] + cy;
    o.v[l] = (uint32_t)s & LMASK;
    cy = s >> LBITS;
  }
  o.v[NL - 1] = (uint32_t)(r.u1 * (int32_t)a.v[NL - 1] + r.u2 * (int32_t)b.v[NL - 1] + r.k * (int32_t)P_[NL - 1] + cy);
  return o;
}

// the recipes of tm_sqr_part8's operands for lane (c, q)
BGV_HD void tm_sqr_rec8(int c, int q, tm_lin_t* X, tm_lin_t* Y) {
  const int k = c >> 1, e = c & 1;
  const uint32_t kI[6] = {0x321, 0x320, 0x430, 0x410, 0x510, 0x210};
  const uint32_t kJ[6] = {0x345, 0x451, 0x452, 0x523, 0x534, 0x345};
  const uint32_t kW[6] = {0x7, 0x6, 0x6, 0x4, 0x4, 0x0};
  if (q < 6) {
    const int p = q >> 1;
    const int i = (kI[k] >> (4 * p)) & 0xf, j = (kJ[k] >> (4 * p)) & 0xf;
    const bool wrap = (kW[k] >> p) & 1, cross = i != j;
    const tm_lin_t y0 = {2 * j, 2 * j, 1, 0, 0}, y1 = {2 * j + 1, 2 * j + 1, 1, 0, 0};
    const tm_lin_t d = {2 * j, 2 * j + 1, 1, -1, 2}, s = {2 * j, 2 * j + 1, 1, 1, 0};
    const int m = cross ? 2 : 1;  // a cross pair's x operand doubled (fp_select(c, a, b) = c ? b : a)
    if ((q & 1) == 0) {
      *X = {2 * i, 2 * i, m, 0, 0};
      *Y = wrap ? (e ? s : d) : (e ? y1 : y0);
    } else {
      *X = e ? tm_lin_t{2 * i + 1, 2 * i + 1, m, 0, 0} : tm_lin_t{2 * i + 1, 2 * i + 1, -m, 0, 2 * m};
      *Y = wrap ? (e ? d : s) : (e ? y0 : y1);
    }
  } else if (q == 6 && (k & 1) == 0) {  // the unwrapped diagonal of even k
    const int h = k >> 1;
    *X = e ? tm_lin_t{2 * h, 2 * h, 2, 0, 0} : tm_lin_t{2 * h, 2 * h + 1, 1, 1, 0};
    *Y = e ? tm_lin_t{2 * h + 1, 2 * h + 1, 1, 0, 0} : tm_lin_t{2 * h, 2 * h + 1, 1, -1, 2};
  } else {  // a zero product
    *X = {0, 0, 0, 0, 0};
    *Y = {0, 0, 1, 0, 0};
  }
}

BGV_HD fp_t tm_sqr_part8_lean(const fp_t* A, const tm_lin_t& X, const tm_lin_t& Y) {
  uint64_t t[2 * NL];
  BGV_UNROLL for (int z = 0; z < 2 * NL; ++z) t[z] = 0;
  wide_mac(t, tm_lin(A, X), tm_lin(A, Y));
  return wide_redc(t);
}

// The four-part squaring (tm_sqr_part) from the same recipes: part q < 3 is pair q's two
// products (eight-part recipes 2q, 2q + 1), part 3 the diagonal (recipes 6, 7).
BGV_HD void tm_sqr_rec4(int c, int q, tm_lin_t* X1, tm_lin_t* Y1, tm_lin_t* X2, tm_lin_t* Y2) {
  tm_sqr_rec8(c, 2 * q, X1, Y1);
  tm_sqr_rec8(c, 2 * q + 1, X2, Y2);
}

BGV_HD fp_t tm_sqr_part4_lean(const fp_t* A, const tm_lin_t& X1, const tm_lin_t& Y1, const tm_lin_t& X2,
                              const tm_lin_t& Y2) {
  uint64_t t[2 * NL];
  BGV_UNROLL for (int z = 0; z < 2 * NL; ++z) t[z] = 0;
  wide_mac(t, tm_lin(A, X1), tm_lin(A, Y1));
  wide_mac(t, tm_lin(A, X2), tm_lin(A, Y2));
  return wide_redc(t);
}

BGV_HD fp_t tm_mul_line_part8(int c, int q, const fp_t* A, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
  const int k = c >> 1, e = c & 1;
  uint64_t t[2 * NL];
  BGV_UNROLL for (int z = 0; z < 2 * NL; ++z) t[z] = 0;
  const int term = q < 6 ? q >> 1 : 0;
  const int j = term == 0 ? 0 : term + 1;  // 0, 2, 3
  const fp2_t& y = term == 0 ? l0 : (term == 1 ? l1 : l3);
  const bool wrap = k < j;
  const int i = wrap ? k - j + 6 : k - j;
  const fp_t x0 = A[2 * i], x1 = A[2 * i + 1];
  const fp_t d = fp_sub_nr(y.c0, y.c1);
  const fp_t s = fp_add_norm(y.c0, y.c1);
  const fp_t x1n = fp_sub_nr(fp_zero(), x1);
  const fp_t X2 = fp_select(e != 0, x1n, x1);
  const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y.c0, y.c1);
  const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y.c1, y.c0);
  const fp_t z = fp_zero();
  wide_mac(t, q < 6 ? ((q & 1) ? X2 : x0) : z, (q & 1) ? Y2 : Y1);
  return wide_redc(t);
}

// a limb-wise sum of four parts (value < 8p, limbs < 2^30) back below 2p: one signed chain
// subtracting q p, q from the top limb (lz_out)
BGV_HD fp_t tm_norm4(const fp_t& r) {
  const uint32_t P_[NL] = BGV_P_LIMBS;
  const uint32_t qt = r.v[NL - 1] / (uint32_t)(P_[NL - 1] + 1);
  int64_t cy = 0;
  fp_t o;
  BGV_UNROLL for (int i = 0; i < NL - 1; ++i) {
    const int64_t s = (int64_t)r.v[i] - (int64_t)((uint64_t)qt * P_[i]) + cy;
    o.v[i] = (uint32_t)s & LMASK;
    cy = s >> LBITS;
  }
  o.v[NL - 1] = (uint32_t)((int64_t)r.v[NL - 1] - (int64_t)((uint64_t)qt * P_[NL - 1]) + cy);
  return o;
}

// sum of the four parts of a coefficient, back below 2p
BGV_HD fp_t tm_sum4(const fp_t& a, const fp_t& b, const fp_t& c, const fp_t& d) {
  fp_t r;
  BGV_UNROLL for (int i = 0; i < NL; ++i) r.v[i] = a.v[i] + b.v[i] + c.v[i] + d.v[i];
  return tm_norm4(r);
}

// sum of the eight parts of a coefficient (each < 1.07 p, limbs < 2^28.1), back below 2p by
// the same one-chain subtraction of qt p (value < 8.6 p, limbs < 2^31.2)
BGV_HD fp_t tm_sum8(const fp_t* x) {
  fp_t r;
  BGV_UNROLL for (int i = 0; i < NL; ++i)
    r.v[i] = x[0].v[i] + x[1].v[i] + x[2].v[i] + x[3].v[i] + x[4].v[i] + x[5].v[i] + x[6].v[i] + x[7].v[i];
  const uint32_t P_[NL] = BGV_P_LIMBS;
  const uint32_t qt = r.v[NL - 1] / (uint32_t)(P_[NL - 1] + 1);
  int64_t cy = 0;
  fp_t o;
  BGV_UNROLL for (int i = 0; i < NL - 1; ++i) {
    const int64_t s = (int64_t)r.v[i] - (int64_t)((uint64_t)qt * P_[i]) + cy;
    o.v[i] = (uint32_t)s & LMASK;
    cy = s >> LBITS;
  }
  o.v[NL - 1] = (uint32_t)((int64_t)r.v[NL - 1] - (int64_t)((uint64_t)qt * P_[NL - 1]) + cy);
  return o;
}

// Frobenius (p-power) on the component pair (x0, x1) = f_k:
// frob(f)_k = conj(f_k) * g_k, g = BGV_FROB1 indexed by tower position.
BGV_HD fp_t tm_frob_lane(int c, const fp_t& x0, const fp_t& x1, const fp2_t& g) {
  const int e = c & 1;
  uint64_t t[2 * NL];
  BGV_UNROLL for (int q = 0; q < 2 * NL; ++q) t[q] = 0;
  // (x0 - x1 u)(g0 + g1 u) = (x0 g0 + x1 g1) + (x0 g1 - x1 g0) u
  wide_mac(t, x0, fp_select(e != 0, g.c0, g.c1));
  wide_mac(t, fp_select(e != 0, x1, fp_sub_nr(fp_zero(), x1)), fp_select(e != 0, g.c1, g.c0));
  return wide_redc(t);
}

BGV_HD int tm_tower_pos(int c) {
  const int k = c >> 1;
  return (k & 1) * 3 + (k >> 1);
}

// A Miller-loop line l = l0 + l1 w^2 + l3 w^3 (bls_pairing.h: tower c0.c0, c0.c1, c1.c1).
// Component c of the line itself (the first step's f = 1 * line).
BGV_HD fp_t tm_line_lane(int c, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
  const int k = c >> 1, e = c & 1;
  const fp2_t& l = k == 0 ? l0 : (k == 2 ? l1 : l3);
  const fp_t v = e ? l.c1 : l.c0;
  return (k == 0 || k == 2 || k == 3) ? v : fp_zero();
}

// Component c = 2k + e of f * l (A: f's 12 w-basis components; the line's three Fp2
// coefficients are held by every lane).  c_k = sum_{j in {0,2,3}} f_{k-j} l_j, xi-scaled
// when k - j wraps below 0: 3 Fp2 terms = 6 double-width products and one reduction
// (tm_mul_lane's formula per term).  Bounds: 6 products < 48 p^2, columns < 2^63.
BGV_HD fp_t tm_mul_line_lane(int c, const fp_t* A, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
  const int k = c >> 1, e = c & 1;
  uint64_t t[2 * NL];
  BGV_UNROLL for (int q = 0; q < 2 * NL; ++q) t[q] = 0;
  BGV_UNROLL for (int term = 0; term < 3; ++term) {
    const int j = term == 0 ? 0 : term + 1;  // 0, 2, 3
    const fp2_t& y = term == 0 ? l0 : (term == 1 ? l1 : l3);
    const bool wrap = k < j;
    const int i = wrap ? k - j + 6 : k - j;
    const fp_t x0 = A[2 * i], x1 = A[2 * i + 1];
    const fp_t d = fp_sub_nr(y.c0, y.c1);
    const fp_t s = fp_add_norm(y.c0, y.c1);
    const fp_t x1n = fp_sub_nr(fp_zero(), x1);
    const fp_t X2 = fp_select(e != 0, x1n, x1);
    const fp_t Y1 = wrap ? fp_select(e != 0, d, s) : fp_select(e != 0, y.c0, y.c1);
    const fp_t Y2 = wrap ? fp_select(e != 0, s, d) : fp_select(e != 0, y.c1, y.c0);
    wide_mac(t, x0, Y1);
    wide_mac(t, X2, Y2);
  }
  return wide_redc(t);
}

// f_{|x|,Q}(P), conjugated (x < 0), with f held by a team: the twist point T and the
// lines are computed by every lane of the team (lane-uniform control flow), the Fp12
// accumulator is coefficient-parallel (O::sqr, O::mul_line).  P and Q Jacobian and
// finite.  Same steps and lines as miller_loop1 (bls_pairing.h), so the value is equal.
template <class E, class O>
BGV_HD E tm_miller_loop(O& o, const g1_jac& p, const g2_jac& q) {
  const miller_p P = miller_p_make(p);
  const miller_jq cq = miller_jq_make(q, P);
  g2_jac t = q;
  fp2_t l0, l1, l3;
  const uint64_t X = BGV_X_ABS;
  miller_dbl(t, &l0, &l1, &l3, P);
  E f = o.line(l0, l1, l3);
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if ((X >> (i + 1)) & 1) {
      miller_add_jq(t, &l0, &l1, &l3, cq);
      f = o.mul_line(f, l0, l1, l3);
    }
    f = o.sqr(f);
    miller_dbl(t, &l0, &l1, &l3, P);
    f = o.mul_line(f, l0, l1, l3);
  }
  return o.conj(f);
}

// The hard-part x-chain on representatives modulo Fp6* (see the header).  O supplies
// mul, sqr, conj, frob, frob2, is_fp6 on its element type E.
template <class O, class E>
BGV_HD E tm_pow_x(O& o, const E& a) {
  const uint64_t X = BGV_X_ABS;
  E r = a;
  BGV_NO_UNROLL for (int i = 62; i >= 0; --i) {
    r = o.sqr(r);
    if ((X >> i) & 1) r = o.mul(r, a);
  }
  return o.conj(r);  // x < 0
}

// u = f^((p^2 + 1) 3 (p^4 - p^2 + 1) / r): the final exponentiation without its (p^6 - 1)
// factor, whose inversion it avoids.  f^(final exp) = u^(p^6 - 1) = conj(u) / u, so the
// pairing value is 1 iff u lies in Fp6 (conj(u) = u).
template <class O, class E>
BGV_HD E tm_final_exp_u(O& o, const E& f) {
  const E t = o.mul(o.frob2(f), f);               // f^(p^2 + 1)
  E a = o.mul(tm_pow_x(o, t), o.conj(t));         // t^(x-1)
  a = o.mul(tm_pow_x(o, a), o.conj(a));           // t^((x-1)^2)
  a = o.mul(tm_pow_x(o, a), o.frob(a));           // ^(x+p)
  E b = tm_pow_x(o, tm_pow_x(o, a));              // a^(x^2)
  b = o.mul(o.mul(b, o.frob2(a)), o.conj(a));     // a^(x^2 + p^2 - 1)
  const E t3 = o.mul(o.sqr(t), t);                // t^3
  return o.mul(b, t3);
}

template <class O, class E>
BGV_HD bool tm_final_exp_is_one(O& o, const E& f) {
  return o.is_fp6(tm_final_exp_u(o, f));
}

// Host emulation of a team (tests): all 12 components in one value, every op
// runs the lane functions above for each lane.
struct tm_emu_t {
  fp_t c[BGV_TEAM_COMPS];
};

struct tm_emu_ops {
  BGV_HD tm_emu_t mul(const tm_emu_t& a, const tm_emu_t& b) {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c) r.c[c] = tm_mul_lane(c, a.c, b.c);
    return r;
  }
  BGV_HD tm_emu_t sqr(const tm_emu_t& a) {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c) r.c[c] = tm_sqr_lane(c, a.c);
    return r;
  }
  BGV_HD tm_emu_t line(const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c) r.c[c] = tm_line_lane(c, l0, l1, l3);
    return r;
  }
  BGV_HD tm_emu_t mul_line(const tm_emu_t& a, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c) r.c[c] = tm_mul_line_lane(c, a.c, l0, l1, l3);
    return r;
  }
  BGV_HD tm_emu_t one() {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c) r.c[c] = c == 0 ? fp_one() : fp_zero();
    return r;
  }
  BGV_HD tm_emu_t conj(const tm_emu_t& a) {
    tm_emu_t r = a;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c)
      if ((c >> 1) & 1) r.c[c] = fp_neg(a.c[c]);
    return r;
  }
  BGV_HD tm_emu_t frob(const tm_emu_t& a) {
    const fp2_t g[6] = BGV_FROB1;
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c)
      r.c[c] = tm_frob_lane(c, a.c[c & ~1], a.c[c | 1], g[tm_tower_pos(c)]);
    return r;
  }
  BGV_HD tm_emu_t frob2(const tm_emu_t& a) {
    const fp_t g[6] = BGV_FROB2;
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c) r.c[c] = fp_mul(a.c[c], g[tm_tower_pos(c)]);
    return r;
  }
  BGV_HD bool is_fp6(const tm_emu_t& a) {
    bool z = true;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c)
      if ((c >> 1) & 1) z = z && fp_is_zero(a.c[c]);
    return z;
  }
};

// the wide products (four parts per coefficient, tm_mul_part / tm_sqr_part), lane by lane
struct tm_emu_wide_ops : tm_emu_ops {
  BGV_HD tm_emu_t mul(const tm_emu_t& a, const tm_emu_t& b) {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c)
      r.c[c] = tm_sum4(tm_mul_part(c, 0, a.c, b.c), tm_mul_part(c, 1, a.c, b.c), tm_mul_part(c, 2, a.c, b.c),
                       tm_mul_part(c, 3, a.c, b.c));
    return r;
  }
  BGV_HD tm_emu_t sqr(const tm_emu_t& a) {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c)
      r.c[c] = tm_sum4(tm_sqr_part(c, 0, a.c), tm_sqr_part(c, 1, a.c), tm_sqr_part(c, 2, a.c), tm_sqr_part(c, 3, a.c));
    return r;
  }
  BGV_HD tm_emu_t mul_line(const tm_emu_t& a, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c)
      r.c[c] = tm_sum4(tm_mul_line_part(c, 0, a.c, l0, l1, l3), tm_mul_line_part(c, 1, a.c, l0, l1, l3),
                       tm_mul_line_part(c, 2, a.c, l0, l1, l3), tm_mul_line_part(c, 3, a.c, l0, l1, l3));
    return r;
  }
};

// the eight-part products (tm_mul_part8 / tm_sqr_part8 / tm_mul_line_part8), lane by lane
struct tm_emu_wide8_ops : tm_emu_ops {
  template <class F>
  BGV_HD tm_emu_t gather8(F part) {
    tm_emu_t r;
    for (int c = 0; c < BGV_TEAM_COMPS; ++c) {
      fp_t x[8];
      for (int q = 0; q < 8; ++q) x[q] = part(c, q);
      r.c[c] = tm_sum8(x);
    }
    return r;
  }
  BGV_HD tm_emu_t mul(const tm_emu_t& a, const tm_emu_t& b) {
    return gather8([&](int c, int q) { return tm_mul_part8(c, q, a.c, b.c); });
  }
  BGV_HD tm_emu_t sqr(const tm_emu_t& a) {
    return gather8([&](int c, int q) { return tm_sqr_part8(c, q, a.c); });
  }
  BGV_HD tm_emu_t mul_line(const tm_emu_t& a, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
    return gather8([&](int c, int q) { return tm_mul_line_part8(c, q, a.c, l0, l1, l3); });
  }
};

// the same with the lean squaring (tm_sqr_rec8 / tm_sqr_part8_lean)
struct tm_emu_wide8_lean_ops : tm_emu_wide8_ops {
  BGV_HD tm_emu_t sqr(const tm_emu_t& a) {
    return gather8([&](int c, int q) {
      tm_lin_t X, Y;
      tm_sqr_rec8(c, q, &X, &Y);
      return tm_sqr_part8_lean(a.c, X, Y);
    });
  }
};

BGV_HD tm_emu_t tm_emu_from_fp12(const fp12_t& f) {
  const fp_t* v = reinterpret_cast<const fp_t*>(&f);
  tm_emu_t r;
  for (int c = 0; c < BGV_TEAM_COMPS; ++c) r.c[c] = v[tm_fp_index(c)];
  return r;
}

BGV_HD fp12_t tm_emu_to_fp12(const tm_emu_t& a) {
  fp12_t f;
  fp_t* v = reinterpret_cast<fp_t*>(&f);
  for (int c = 0; c < BGV_TEAM_COMPS; ++c) v[tm_fp_index(c)] = a.c[c];
  return f;
}
