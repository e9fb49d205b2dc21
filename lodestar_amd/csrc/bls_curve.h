// G1 / G2 group arithmetic on CDNA4, one point per lane.
//
// E1: y^2 = x^3 + 4 over Fp;  E2: y^2 = x^3 + 4(1+i) over Fp2.
// Points are Jacobian (X, Y, Z), x = X/Z^2, y = Y/Z^3, infinity <=> Z == 0.
// Formulas: dbl-2009-l, add-2007-bl, madd-2007-bl (a = 0), made complete with
// rare-case branches (equal inputs -> double, infinity operands).
#pragma once
#include "bls_field.h"
#include "bls_lazy.h"

// ---------------------------------------------------------------------------
// overload set so the point code is written once for Fp and Fp2
// ---------------------------------------------------------------------------
BGV_HD fp_t f_add(const fp_t& a, const fp_t& b) { return fp_add(a, b); }
BGV_HD fp_t f_sub(const fp_t& a, const fp_t& b) { return fp_sub(a, b); }
BGV_HD fp_t f_dbl(const fp_t& a) { return fp_dbl(a); }
BGV_HD fp_t f_neg(const fp_t& a) { return fp_neg(a); }
BGV_HD fp_t f_mul(const fp_t& a, const fp_t& b) { return fp_mul(a, b); }
BGV_HD fp_t f_sqr(const fp_t& a) { return fp_sqr(a); }
BGV_HD bool f_is_zero(const fp_t& a) { return fp_is_zero(a); }
BGV_HD bool f_eq(const fp_t& a, const fp_t& b) { return fp_eq(a, b); }
BGV_HD fp_t f_select(bool c, const fp_t& a, const fp_t& b) { return fp_select(c, a, b); }
BGV_HD fp_t f_inv(const fp_t& a) { return fp_inv(a); }
BGV_HD void f_set_zero(fp_t* a) { *a = fp_zero(); }
BGV_HD void f_set_one(fp_t* a) { *a = fp_one(); }

BGV_HD fp2_t f_add(const fp2_t& a, const fp2_t& b) { return fp2_add(a, b); }
BGV_HD fp2_t f_sub(const fp2_t& a, const fp2_t& b) { return fp2_sub(a, b); }
BGV_HD fp2_t f_dbl(const fp2_t& a) { return fp2_dbl(a); }
BGV_HD fp2_t f_neg(const fp2_t& a) { return fp2_neg(a); }
BGV_HD fp2_t f_mul(const fp2_t& a, const fp2_t& b) { return fp2_mul(a, b); }
BGV_HD fp2_t f_sqr(const fp2_t& a) { return fp2_sqr(a); }
BGV_HD bool f_is_zero(const fp2_t& a) { return fp2_is_zero(a); }
BGV_HD bool f_eq(const fp2_t& a, const fp2_t& b) { return fp2_eq(a, b); }
BGV_HD fp2_t f_select(bool c, const fp2_t& a, const fp2_t& b) { return fp2_select(c, a, b); }
BGV_HD fp2_t f_inv(const fp2_t& a) { return fp2_inv(a); }
BGV_HD void f_set_zero(fp2_t* a) { *a = fp2_zero(); }
BGV_HD void f_set_one(fp2_t* a) { *a = fp2_one(); }

template <class F>
struct jac_t {
  F x, y, z;
};
template <class F>
struct aff_t {
  F x, y;
};

typedef jac_t<fp_t> g1_jac;
typedef aff_t<fp_t> g1_aff;
typedef jac_t<fp2_t> g2_jac;
typedef aff_t<fp2_t> g2_aff;

template <class F>
BGV_HD jac_t<F> jac_infinity() {
  jac_t<F> r;
  f_set_one(&r.x);
  f_set_one(&r.y);
  f_set_zero(&r.z);
  return r;
}

template <class F>
BGV_HD bool jac_is_inf(const jac_t<F>& p) {
  return f_is_zero(p.z);
}

template <class F>
BGV_HD jac_t<F> jac_from_aff(const aff_t<F>& a) {
  jac_t<F> r;
  r.x = a.x;
  r.y = a.y;
  f_set_one(&r.z);
  return r;
}

template <class F>
BGV_HD jac_t<F> jac_select(bool c, const jac_t<F>& a, const jac_t<F>& b) {
  return jac_t<F>{f_select(c, a.x, b.x), f_select(c, a.y, b.y), f_select(c, a.z, b.z)};
}

template <class F>
BGV_HD jac_t<F> jac_neg(const jac_t<F>& p) {
  return jac_t<F>{p.x, f_neg(p.y), p.z};
}

// Jacobian doubling/addition are inlined into their callers: the scalar-multiplication
// loops ([x]P for the G2 subgroup check and cofactor clearing, r * pk) keep the point in
// VGPRs instead of passing it through scratch on every step (k_prep 31.0 -> 29.4 ms per
// 131,072 sets with the eager formulas).
#define BGV_CURVE_ATTR BGV_HD

// dbl-2009-l on lazy values (bls_lazy.h): E = 3A, F = E^2 = 9 A^2; the same field elements
// as the eager formulas, each output reduced once (< 2p)
template <class F>
BGV_CURVE_ATTR jac_t<F> jac_dbl(const jac_t<F>& p) {
  const auto X = L_in(p.x), Y = L_in(p.y), Z = L_in(p.z);
  const auto A = L_sqr(X);
  const auto B = L_sqr(Y);
  const auto C = L_sqr(B);
  const auto D = L_norm(L_dbl(L_sub(L_sqr(L_norm(L_add(X, B))), L_add(A, C))));
  const auto X3 = L_norm(L_sub(L_mulk<9>(L_sqr(A)), L_dbl(D)));
  const auto Y3 = L_sub(L_mulk<3>(L_mul(A, L_norm(L_sub(D, X3)))), L_mulk<8>(C));
  jac_t<F> r;
  r.x = L_out(X3);
  r.y = L_out(Y3);
  r.z = L_out(L_dbl(L_mul(Y, Z)));
  return r;
}

// add-2007-bl with the generic-case formulas (I = (2H)^2 = 4 HH, J = H I, V = U1 I);
// flags equal/opposite inputs.
template <class F>
BGV_HD jac_t<F> jac_add_raw(const jac_t<F>& p, const jac_t<F>& q, bool* h_zero, bool* r_zero) {
  const auto X1 = L_in(p.x), Y1 = L_in(p.y), Z1 = L_in(p.z);
  const auto X2 = L_in(q.x), Y2 = L_in(q.y), Z2 = L_in(q.z);
  const auto Z1Z1 = L_sqr(Z1);
  const auto Z2Z2 = L_sqr(Z2);
  const auto U1 = L_mul(X1, Z2Z2);
  const auto U2 = L_mul(X2, Z1Z1);
  const auto S1 = L_mul(L_mul(Y1, Z2), Z2Z2);
  const auto S2 = L_mul(L_mul(Y2, Z1), Z1Z1);
  const auto H = L_norm(L_sub(U2, U1));
  const auto HH = L_sqr(H);
  const auto J = L_mulk<4>(L_mul(H, HH));
  const auto rr = L_red(L_dbl(L_sub(S2, S1)));
  const auto V = L_mulk<4>(L_mul(U1, HH));
  const auto X3 = L_norm(L_sub(L_sqr(rr), L_add(J, L_dbl(V))));
  const auto Y3 = L_sub(L_mul(rr, L_norm(L_sub(V, X3))), L_dbl(L_mul(S1, L_norm(J))));
  const auto Z3 = L_mul(L_wnorm(L_sub(L_sqr(L_norm(L_add(Z1, Z2))), L_add(Z1Z1, Z2Z2))), H);
  jac_t<F> r;
  r.x = L_out(X3);
  r.y = L_out(Y3);
  r.z = L_out(Z3);
  *h_zero = L_is_zero(H);
  *r_zero = L_is_zero(rr);
  return r;
}

// complete addition
template <class F>
BGV_CURVE_ATTR jac_t<F> jac_add(const jac_t<F>& p, const jac_t<F>& q) {
  bool hz, rz;
  jac_t<F> r = jac_add_raw(p, q, &hz, &rz);
  const bool pinf = jac_is_inf(p), qinf = jac_is_inf(q);
  if (hz && rz && !pinf && !qinf) r = jac_dbl(p);  // rare: P == Q
  r = jac_select(pinf, r, q);
  r = jac_select(qinf && !pinf, r, p);
  return r;
}

// madd-2007-bl: p Jacobian + q affine (q never infinity), lazy values as in jac_add_raw
template <class F>
BGV_HD jac_t<F> jac_add_aff_raw(const jac_t<F>& p, const aff_t<F>& q, bool* h_zero, bool* r_zero) {
  const auto X1 = L_in(p.x), Y1 = L_in(p.y), Z1 = L_in(p.z);
  const auto X2 = L_in(q.x), Y2 = L_in(q.y);
  const auto Z1Z1 = L_sqr(Z1);
  const auto U2 = L_mul(X2, Z1Z1);
  const auto S2 = L_mul(Y2, L_mul(Z1, Z1Z1));
  const auto H = L_norm(L_sub(U2, X1));
  const auto HH = L_sqr(H);
  const auto J = L_mulk<4>(L_mul(H, HH));
  const auto rr = L_red(L_dbl(L_sub(S2, Y1)));
  const auto V = L_mulk<4>(L_mul(X1, HH));
  const auto X3 = L_norm(L_sub(L_sqr(rr), L_add(J, L_dbl(V))));
  const auto Y3 = L_sub(L_mul(rr, L_norm(L_sub(V, X3))), L_dbl(L_mul(Y1, L_norm(J))));
  const auto Z3 = L_sub(L_sqr(L_norm(L_add(Z1, H))), L_add(Z1Z1, HH));
  jac_t<F> r;
  r.x = L_out(X3);
  r.y = L_out(Y3);
  r.z = L_out(Z3);
  *h_zero = L_is_zero(H);
  *r_zero = L_is_zero(rr);
  return r;
}

template <class F>
BGV_NOINLINE jac_t<F> jac_add_aff(const jac_t<F>& p, const aff_t<F>& q) {
  bool hz, rz;
  jac_t<F> r = jac_add_aff_raw(p, q, &hz, &rz);
  const bool pinf = jac_is_inf(p);
  if (hz && rz && !pinf) r = jac_dbl(p);
  r = jac_select(pinf, r, jac_from_aff(q));
  return r;
}

// Jacobian -> affine; returns false for infinity (out untouched = zeros).
template <class F>
BGV_NOINLINE bool jac_to_aff(aff_t<F>* out, const jac_t<F>& p) {
  F zi = f_inv(p.z);
  F zi2 = f_sqr(zi);
  out->x = f_mul(p.x, zi2);
  out->y = f_mul(p.y, f_mul(zi2, zi));
  return !jac_is_inf(p);
}

// Two finite Jacobian points -> affine with one shared inversion.
template <class F>
BGV_NOINLINE void jac2_to_aff(aff_t<F>* a, aff_t<F>* b, const jac_t<F>& p, const jac_t<F>& q) {
  const F zi = f_inv(f_mul(p.z, q.z));
  const F pzi = f_mul(zi, q.z), qzi = f_mul(zi, p.z);
  F t = f_sqr(pzi);
  a->x = f_mul(p.x, t);
  a->y = f_mul(p.y, f_mul(t, pzi));
  t = f_sqr(qzi);
  b->x = f_mul(q.x, t);
  b->y = f_mul(q.y, f_mul(t, qzi));
}

template <class F>
BGV_HD bool jac_eq(const jac_t<F>& p, const jac_t<F>& q) {
  const bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  F Z1Z1 = f_sqr(p.z), Z2Z2 = f_sqr(q.z);
  bool ex = f_eq(f_mul(p.x, Z2Z2), f_mul(q.x, Z1Z1));
  bool ey = f_eq(f_mul(f_mul(p.y, q.z), Z2Z2), f_mul(f_mul(q.y, p.z), Z1Z1));
  return (pi && qi) || (!pi && !qi && ex && ey);
}

// An index the compiler cannot fold (always 0): reading a point through tab[bgv_opaque0()]
// keeps it in (scratch) memory, read where it is used, instead of live in registers across
// a loop that has no room for it -- in which case the allocator spills it on every
// iteration (k_prep: ~650 KB of scratch traffic per set before, tools/gpu notes in DESIGN).
BGV_HD int bgv_opaque0() {
  int z = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(z));
#else
  asm volatile("" : "+r"(z));
#endif
  return z;
}

// [k]P for a 64-bit (lane-varying) scalar: left-to-right fixed window of BGV_MUL_WINDOW
// bits over the table P, 2P, ..., (2^w - 1)P; the add is computed in every lane and
// selected, so a wave never diverges on scalar bits.  The table lives in memory and one
// entry is loaded per window (the accumulator and the addition's temporaries fill the
// registers).
#ifndef BGV_MUL_WINDOW
#define BGV_MUL_WINDOW 3
#endif
template <class F>
BGV_NOINLINE jac_t<F> jac_mul_u64(const jac_t<F>& p, uint64_t k) {
  constexpr int W = BGV_MUL_WINDOW, NT = 1 << W, NWIN = (64 + W - 1) / W;
  jac_t<F> tab[NT];
  tab[1] = p;
  tab[2] = jac_dbl(p);
  BGV_NO_UNROLL for (int i = 3; i < NT; ++i) tab[i] = jac_add(tab[i - 1], p);
  tab[0] = tab[1];
  jac_t<F> acc = jac_infinity<F>();
  BGV_NO_UNROLL for (int j = NWIN - 1; j >= 0; --j) {
    BGV_UNROLL for (int t = 0; t < W; ++t) acc = jac_dbl(acc);
    const uint32_t d = (uint32_t)(k >> (W * j)) & (uint32_t)(NT - 1);
    const jac_t<F> sum = jac_add(acc, tab[d]);
    acc = jac_select(d != 0u, acc, sum);
  }
  return acc;
}

// [k]P for a 256-bit scalar given as 8 little-endian u32 words (secret keys in
// the keygen/sign utilities), same 2-bit fixed window as jac_mul_u64.
template <class F>
BGV_NOINLINE jac_t<F> jac_mul_u256(const jac_t<F>& p, const uint32_t k[8]) {
  jac_t<F> tab[4];
  tab[1] = p;
  tab[2] = jac_dbl(p);
  tab[3] = jac_add(tab[2], p);
  tab[0] = tab[1];
  jac_t<F> acc = jac_infinity<F>();
  BGV_NO_UNROLL for (int i = 254; i >= 0; i -= 2) {
    acc = jac_dbl(jac_dbl(acc));
    const uint32_t d = (k[i >> 5] >> (i & 31)) & 3u;
    const jac_t<F> sum = jac_add(acc, tab[d]);
    acc = jac_select(d != 0u, acc, sum);
  }
  return acc;
}

// [|x|]P, |x| = 0xd201000000010000 (lane-uniform bits: no divergence).  P is read from
// memory at the 5 additions; the 63 doublings keep only the accumulator live.
template <class F>
BGV_NOINLINE jac_t<F> jac_mul_x_abs(const jac_t<F>& p) {
  jac_t<F> pm[1];
  pm[0] = p;
  jac_t<F> acc = p;
  const uint64_t X = BGV_X_ABS;
  BGV_NO_UNROLL for (int i = 62; i >= 0; --i) {
    acc = jac_dbl(acc);
    if ((X >> i) & 1) acc = jac_add(acc, pm[bgv_opaque0()]);
  }
  return jac_t<F>{acc.x, acc.y, acc.z};  // not NRVO: acc would live in the caller's return slot (scratch)
}

// ---------------------------------------------------------------------------
// G1 helpers
// ---------------------------------------------------------------------------
BGV_HD g1_aff g1_generator() {
  g1_aff g;
  g.x = fp_t{BGV_G1X};
  g.y = fp_t{BGV_G1Y};
  return g;
}

BGV_HD g1_aff g1_neg_generator() {
  g1_aff g;
  g.x = fp_t{BGV_G1X};
  g.y = fp_t{BGV_NEG_G1Y};
  return g;
}

BGV_HD bool g1_aff_on_curve(const g1_aff& a) {
  const fp_t b = {BGV_B1};
  return fp_eq(fp_sqr(a.y), fp_add(fp_mul(fp_sqr(a.x), a.x), b));
}

// ---------------------------------------------------------------------------
// G2 helpers: psi endomorphism and subgroup check
// ---------------------------------------------------------------------------
BGV_HD g2_jac g2_psi(const g2_jac& p) {
  const fp2_t cx = BGV_PSI_CX;
  const fp2_t cy = BGV_PSI_CY;
  g2_jac r;
  r.x = fp2_mul(fp2_conj(p.x), cx);
  r.y = fp2_mul(fp2_conj(p.y), cy);
  r.z = fp2_conj(p.z);
  return r;
}

BGV_HD g2_jac g2_psi2(const g2_jac& p) {
  const fp_t cx = {BGV_PSI2_CX};
  const fp_t cy = {BGV_PSI2_CY};
  g2_jac r;
  r.x = fp2_mul_fp(p.x, cx);
  r.y = fp2_mul_fp(p.y, cy);
  r.z = p.z;
  return r;
}

// The batch randomizers (bgv_dslot.scalar) are r = a + b x^2 mod the group order, a and b the
// low and high 32 bits of the 64-bit word (never both zero).  x^2 is an eigenvalue of a cheap
// endomorphism on both groups, so r P = a P + b E(P) costs 32 doublings instead of 64:
//   G1  E(X, Y, Z) = (beta X, -Y, Z): phi(x, y) = (beta x, y) is [-x^2] on G1 for this beta
//   G2  E = psi^2 = [p^2] = [x^2] on G2 (p = x mod the group order)
// The 2^64 - 1 pairs (a, b) give distinct r (|a + b x^2| < 2^160 < the order), so a bad set
// passes the batch equation with probability <= 2^-64, as with blst's 64-bit scalars.
BGV_HD g1_jac jac_endo_x2(const g1_jac& p) {
  const fp_t beta = {BGV_BETA_MX2};
  return g1_jac{fp_mul(p.x, beta), fp_neg(p.y), p.z};
}
BGV_HD g2_jac jac_endo_x2(const g2_jac& p) { return g2_psi2(p); }

// r P with r = lo32(k) + hi32(k) x^2: interleaved 3-bit fixed windows over one table
// T[j] = jP (j < 8, in memory, one entry loaded per window and scalar half), the second
// half's entry mapped through E on the fly; adds computed in every lane and selected, as in
// jac_mul_u64.  Valid for P in the prime-order subgroup (a signature after its subgroup
// check, a cached or aggregated pubkey); P infinity gives infinity.
template <class F>
BGV_NOINLINE jac_t<F> jac_mul_glv(const jac_t<F>& p, uint64_t k) {
  constexpr int W = 3, NT = 1 << W, NWIN = (32 + W - 1) / W;
  const uint32_t a = (uint32_t)k, b = (uint32_t)(k >> 32);
  jac_t<F> tab[NT];
  tab[1] = p;
  tab[2] = jac_dbl(p);
  BGV_NO_UNROLL for (int i = 3; i < NT; ++i) tab[i] = jac_add(tab[i - 1], p);
  tab[0] = tab[1];
  jac_t<F> acc = jac_infinity<F>();
  BGV_NO_UNROLL for (int j = NWIN - 1; j >= 0; --j) {
    BGV_UNROLL for (int t = 0; t < W; ++t) acc = jac_dbl(acc);
    const uint32_t da = (a >> (W * j)) & (uint32_t)(NT - 1);
    const jac_t<F> sa = jac_add(acc, tab[da]);
    acc = jac_select(da != 0u, acc, sa);
    const uint32_t db = (b >> (W * j)) & (uint32_t)(NT - 1);
    const jac_t<F> sb = jac_add(acc, jac_endo_x2(tab[db]));
    acc = jac_select(db != 0u, acc, sb);
  }
  return jac_t<F>{acc.x, acc.y, acc.z};  // not NRVO (see jac_mul_x_abs)
}

BGV_HD bool g2_aff_on_curve(const g2_aff& a) {
  const fp2_t b = BGV_B2;
  return fp2_eq(fp2_sqr(a.y), fp2_add(fp2_mul(fp2_sqr(a.x), a.x), b));
}

// P in G2  <=>  psi(P) == [x]P == -[|x|]P   (Scott, "A note on group membership
// tests for G1, G2 and GT on BLS pairing-friendly curves"; blst POINTonE2_in_G2)
BGV_HD bool g2_in_subgroup(const g2_jac& p) {
  g2_jac q = jac_neg(jac_mul_x_abs(p));
  return jac_eq(g2_psi(p), q);
}

// [x]P with x = -|x|
template <class F>
BGV_HD jac_t<F> jac_mul_x(const jac_t<F>& p) {
  return jac_neg(jac_mul_x_abs(p));
}

// RFC 9380 G.4 clear_cofactor: (x^2 - x - 1)P + (x - 1)psi(P) + 2 psi^2(P)
BGV_HD g2_jac g2_clear_cofactor(const g2_jac& p) {
  g2_jac t1 = jac_mul_x(p);
  g2_jac t2 = g2_psi(p);
  g2_jac t3 = g2_psi2(jac_dbl(p));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_mul_x(t2);
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}

// ---------------------------------------------------------------------------
// ZCash serialisation (big-endian; flags in the top 3 bits of byte 0)
// ---------------------------------------------------------------------------
enum {
  BGV_OK = 0,
  BGV_BAD_ENCODING = 1,
  BGV_POINT_NOT_ON_CURVE = 2,
  BGV_POINT_NOT_IN_GROUP = 3,
  BGV_PK_IS_INFINITY = 6,
  BGV_INVALID_SIZE = 8,
};

// 96-byte compressed G2 (signature) -> affine; *inf set for the infinity
// encoding.  Mirrors blst_p2_uncompress; returns a BGV_* code.  PW: the square root's
// exponentiation policy (bls_field.h bgv_pow_lane / bgv_wfp.h bgv_pow_wave).
template <class PW>
BGV_HD int g2_decompress_t(g2_aff* out, bool* inf, const uint8_t* b) {
  const uint8_t flags = b[0];
  *inf = false;
  if (!(flags & 0x80)) return BGV_BAD_ENCODING;
  if (flags & 0x40) {
    uint8_t acc = flags & 0x3f;
    for (int i = 1; i < 96; ++i) acc |= b[i];
    if (acc) return BGV_BAD_ENCODING;
    *inf = true;
    return BGV_OK;
  }
  uint8_t tmp[48];
  for (int i = 0; i < 48; ++i) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  fp_t x1 = fp_from_be48(tmp);
  fp_t x0 = fp_from_be48(b + 48);
  if (!fp_raw_lt_p(x1) || !fp_raw_lt_p(x0)) return BGV_BAD_ENCODING;
  fp2_t x = {fp_to_mont(x0), fp_to_mont(x1)};
  const fp2_t B = BGV_B2;
  fp2_t y2 = fp2_add(fp2_mul(fp2_sqr(x), x), B);
  fp2_t y;
  if (!fp2_sqrt_t<PW>(&y, y2)) return BGV_POINT_NOT_ON_CURVE;
  const bool want = (flags & 0x20) != 0;
  if (fp2_lex_largest(y) != want) y = fp2_neg(y);
  out->x = x;
  out->y = y;
  return BGV_OK;
}
BGV_HD int g2_decompress(g2_aff* out, bool* inf, const uint8_t* b) { return g2_decompress_t<bgv_pow_lane>(out, inf, b); }

BGV_HD void g2_compress(uint8_t* b, const g2_aff& a, bool inf) {
  if (inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 96; ++i) b[i] = 0;
    return;
  }
  fp_to_be48(b, fp_from_mont(a.x.c1));
  fp_to_be48(b + 48, fp_from_mont(a.x.c0));
  b[0] |= 0x80 | (fp2_lex_largest(a.y) ? 0x20 : 0);
}

BGV_HD void g2_serialize(uint8_t* b, const g2_aff& a, bool inf) {
  if (inf) {
    b[0] = 0x40;
    for (int i = 1; i < 192; ++i) b[i] = 0;
    return;
  }
  fp_to_be48(b, fp_from_mont(a.x.c1));
  fp_to_be48(b + 48, fp_from_mont(a.x.c0));
  fp_to_be48(b + 96, fp_from_mont(a.y.c1));
  fp_to_be48(b + 144, fp_from_mont(a.y.c0));
}

BGV_HD int g1_decompress(g1_aff* out, bool* inf, const uint8_t* b);

// 96-byte G1 record (trusted pubkey bytes, worker.ts:110-116), decoded like blst's
// POINTonE1_Deserialize_Z (PublicKey.fromBytes of 96 bytes): no subgroup check.
//   top bits 000 -> big-endian x || y: x, y < p else BAD_ENCODING; on the curve else
//                   POINT_NOT_ON_CURVE; x == 0 (the points (0, +-2)) -> POINT_NOT_IN_GROUP
//   0x80 set     -> the first 48 bytes as a compressed point
//   0x40 only    -> infinity iff every other bit is zero
//   anything else (0x20 without 0x80 / 0x40) -> BAD_ENCODING
BGV_HD int g1_deserialize(g1_aff* out, bool* inf, const uint8_t* b) {
  const uint8_t flags = b[0];
  *inf = false;
  if (flags & 0x80) return g1_decompress(out, inf, b);
  if (flags & 0x40) {
    uint8_t acc = flags & 0x3f;
    for (int i = 1; i < 96; ++i) acc |= b[i];
    if (acc) return BGV_BAD_ENCODING;
    *inf = true;
    return BGV_OK;
  }
  if (flags & 0x20) return BGV_BAD_ENCODING;
  fp_t x = fp_from_be48(b);
  fp_t y = fp_from_be48(b + 48);
  if (!fp_raw_lt_p(x) || !fp_raw_lt_p(y)) return BGV_BAD_ENCODING;
  out->x = fp_to_mont(x);
  out->y = fp_to_mont(y);
  if (!g1_aff_on_curve(*out)) return BGV_POINT_NOT_ON_CURVE;
  uint32_t nz = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) nz |= x.v[i];
  if (nz == 0) return BGV_POINT_NOT_IN_GROUP;
  return BGV_OK;
}

// 48-byte compressed G1 -> affine (blst_p1_uncompress)
BGV_HD int g1_decompress(g1_aff* out, bool* inf, const uint8_t* b) {
  const uint8_t flags = b[0];
  *inf = false;
  if (!(flags & 0x80)) return BGV_BAD_ENCODING;
  if (flags & 0x40) {
    uint8_t acc = flags & 0x3f;
    for (int i = 1; i < 48; ++i) acc |= b[i];
    if (acc) return BGV_BAD_ENCODING;
    *inf = true;
    return BGV_OK;
  }
  uint8_t tmp[48];
  for (int i = 0; i < 48; ++i) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  fp_t xr = fp_from_be48(tmp);
  if (!fp_raw_lt_p(xr)) return BGV_BAD_ENCODING;
  fp_t x = fp_to_mont(xr);
  const fp_t B = {BGV_B1};
  fp_t y;
  if (!fp_sqrt(&y, fp_add(fp_mul(fp_sqr(x), x), B))) return BGV_POINT_NOT_ON_CURVE;
  if (fp_lex_largest(y) != ((flags & 0x20) != 0)) y = fp_neg(y);
  out->x = x;
  out->y = y;
  // (0, +-2) is on the curve but of order 3: blst's POINTonE1_Uncompress_Z rejects it
  uint32_t nz = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) nz |= xr.v[i];
  return nz ? BGV_OK : BGV_POINT_NOT_IN_GROUP;
}

BGV_HD void g1_serialize(uint8_t* b, const g1_aff& a, bool inf) {
  if (inf) {
    b[0] = 0x40;
    for (int i = 1; i < 96; ++i) b[i] = 0;
    return;
  }
  fp_to_be48(b, fp_from_mont(a.x));
  fp_to_be48(b + 48, fp_from_mont(a.y));
}

BGV_HD void g1_compress(uint8_t* b, const g1_aff& a, bool inf) {
  if (inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 48; ++i) b[i] = 0;
    return;
  }
  fp_to_be48(b, fp_from_mont(a.x));
  b[0] |= 0x80 | (fp_lex_largest(a.y) ? 0x20 : 0);
}
