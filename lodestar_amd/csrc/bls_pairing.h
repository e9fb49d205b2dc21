// Optimal-ate pairing pieces on CDNA4: Miller loop (Jacobian twist point,
// lines evaluated straight into the sparse Fp12 product) and final
// exponentiation (easy part + x-chain hard part computing the cube of the
// pairing, which has the same kernel since gcd(3, r) = 1).
#pragma once
#include <type_traits>

#include "bls_curve.h"
#include "bls_lazy.h"

// The G1 point of a Miller loop in Jacobian form P = (X : Y : Z) (no inversion after
// r_i * pk_i): every line is scaled by Z^3, an Fp factor the final exponentiation kills,
// so xP = X / Z^2 enters as X Z, yP = Y / Z^3 as Y, and the P-free term as l0 Z^3.
struct miller_p {
  fp_t xn;   // -X Z
  fp_t yp;   // Y
  fp_t zp3;  // Z^3
};
BGV_HD miller_p miller_p_make(const g1_jac& p) {
  return miller_p{fp_neg(fp_mul(p.x, p.z)), p.y, fp_mul(fp_sqr(p.z), p.z)};
}
BGV_HD miller_p miller_p_aff(const g1_aff& p) { return miller_p{fp_neg(p.x), p.y, fp_one()}; }

// Doubling step: T <- 2T; returns the tangent line at T evaluated at P,
// scaled by Fp2/Fp4 factors that the final exponentiation kills:
//   l0 = (3X^3 - 2Y^2) Z_P^3,  l1 = -3X^2 Z^2 X_P Z_P,  l3 = Z3 Z^2 Y_P
BGV_MILLER_ATTR void miller_dbl(g2_jac& t, fp2_t* l0, fp2_t* l1, fp2_t* l3, const miller_p& P) {
  const fp_t& xp_neg = P.xn;
  const fp_t& yp = P.yp;
  fp2_t A = fp2_sqr(t.x);
  fp2_t B = fp2_sqr(t.y);
  fp2_t C = fp2_sqr(B);
  fp2_t ZZ = fp2_sqr(t.z);
  fp2_t D = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(t.x, B)), A), C));
  fp2_t E = fp2_add(fp2_dbl(A), A);
  fp2_t F = fp2_sqr(E);
  *l0 = fp2_mul_fp(fp2_sub(fp2_mul(E, t.x), fp2_dbl(B)), P.zp3);
  *l1 = fp2_mul_fp(fp2_mul(E, ZZ), xp_neg);
  fp2_t X3 = fp2_sub(F, fp2_dbl(D));
  fp2_t Y3 = fp2_sub(fp2_mul(E, fp2_sub(D, X3)), fp2_dbl(fp2_dbl(fp2_dbl(C))));
  fp2_t Z3 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(t.y, t.z)), B), ZZ);
  *l3 = fp2_mul_fp(fp2_mul(Z3, ZZ), yp);
  t.x = X3;
  t.y = Y3;
  t.z = Z3;
}

// Addition step: T <- T + Q (Q affine); returns the chord line at P:
//   l0 = r xQ - yQ Z3,  l1 = -r xP,  l3 = Z3 yP   (r = 2(S2 - Y))
BGV_MILLER_ATTR void miller_add(g2_jac& t, fp2_t* l0, fp2_t* l1, fp2_t* l3, const g2_aff& q, const fp_t& xp_neg,
                       const fp_t& yp) {  // P affine (Z_P = 1)
  fp2_t ZZ = fp2_sqr(t.z);
  fp2_t U2 = fp2_mul(q.x, ZZ);
  fp2_t S2 = fp2_mul(q.y, fp2_mul(t.z, ZZ));
  fp2_t H = fp2_sub(U2, t.x);
  fp2_t HH = fp2_sqr(H);
  fp2_t I = fp2_dbl(fp2_dbl(HH));
  fp2_t J = fp2_mul(H, I);
  fp2_t r = fp2_dbl(fp2_sub(S2, t.y));
  fp2_t V = fp2_mul(t.x, I);
  fp2_t X3 = fp2_sub(fp2_sub(fp2_sqr(r), J), fp2_dbl(V));
  fp2_t Y3 = fp2_sub(fp2_mul(r, fp2_sub(V, X3)), fp2_dbl(fp2_mul(t.y, J)));
  fp2_t Z3 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(t.z, H)), ZZ), HH);
  *l0 = fp2_sub(fp2_mul(r, q.x), fp2_mul(q.y, Z3));
  *l1 = fp2_mul_fp(r, xp_neg);
  *l3 = fp2_mul_fp(Z3, yp);
  t.x = X3;
  t.y = Y3;
  t.z = Z3;
}

// f_{|x|,Q}(P), conjugated for x < 0.  P = (xP, yP) in G1, Q in G2, both affine
// and not infinity.  Loop over the bits of |x| = 0xd201000000010000 below the top.
BGV_NOINLINE fp12_t miller_loop(const g1_aff& p, const g2_aff& q) {
  const fp_t xp_neg = fp_neg(p.x);
  const fp_t yp = p.y;
  const miller_p P = miller_p_aff(p);
  g2_jac t = jac_from_aff(q);
  fp12_t f = fp12_one();
  fp2_t l0, l1, l3;
  const uint64_t X = BGV_X_ABS;
  // first doubling: f = 1, so f^2 * line = line
  miller_dbl(t, &l0, &l1, &l3, P);
  f = fp12_mul_line(f, l0, l1, l3);
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if ((X >> (i + 1)) & 1) {
      miller_add(t, &l0, &l1, &l3, q, xp_neg, yp);
      f = fp12_mul_line(f, l0, l1, l3);
    }
    f = fp12_sqr(f);
    miller_dbl(t, &l0, &l1, &l3, P);
    f = fp12_mul_line(f, l0, l1, l3);
  }
  // bit 0 of |x| is 0: no trailing addition
  return fp12_conj(f);
}

// Addition step with a Jacobian Q = (X2 : Y2 : Z2) (no affine conversion of Q):
// T <- T + Q, and the chord line at P scaled by Z2^3 (an Fp2 factor) and Z_P^3 (Fp), both
// killed by the final exponentiation:  l0 = (r X2 Z2 - Y2 Z3) Z_P^3,  l1 = -r Z2^3 X_P Z_P,
// l3 = Z3 Z2^3 Y_P.  Per-pair constants: q.zz = Z2^2, q.xz = X2 Z2 Z_P^3, q.y2z = Y2 Z_P^3,
// q.zzz_xn = -Z2^3 X_P Z_P, q.zzz_yp = Z2^3 Y_P.
struct miller_jq {
  g2_jac q;
  fp2_t zz, xz, y2z, zzz_xn, zzz_yp;
};

BGV_HD miller_jq miller_jq_make(const g2_jac& q, const miller_p& P) {
  miller_jq r;
  r.q = q;
  r.zz = fp2_sqr(q.z);
  const fp2_t zzz = fp2_mul(r.zz, q.z);
  r.xz = fp2_mul_fp(fp2_mul(q.x, q.z), P.zp3);
  r.y2z = fp2_mul_fp(q.y, P.zp3);
  r.zzz_xn = fp2_mul_fp(zzz, P.xn);
  r.zzz_yp = fp2_mul_fp(zzz, P.yp);
  return r;
}

BGV_MILLER_ATTR void miller_add_jq(g2_jac& t, fp2_t* l0, fp2_t* l1, fp2_t* l3, const miller_jq& c) {
  fp2_t ZZ = fp2_sqr(t.z);
  fp2_t U1 = fp2_mul(t.x, c.zz);
  fp2_t U2 = fp2_mul(c.q.x, ZZ);
  fp2_t S1 = fp2_mul(t.y, fp2_mul(c.zz, c.q.z));
  fp2_t S2 = fp2_mul(c.q.y, fp2_mul(t.z, ZZ));
  fp2_t H = fp2_sub(U2, U1);
  fp2_t HH = fp2_sqr(H);
  fp2_t I = fp2_dbl(fp2_dbl(HH));
  fp2_t J = fp2_mul(H, I);
  fp2_t r = fp2_dbl(fp2_sub(S2, S1));
  fp2_t V = fp2_mul(U1, I);
  fp2_t X3 = fp2_sub(fp2_sub(fp2_sqr(r), J), fp2_dbl(V));
  fp2_t Y3 = fp2_sub(fp2_mul(r, fp2_sub(V, X3)), fp2_dbl(fp2_mul(S1, J)));
  fp2_t Z3 = fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(t.z, c.q.z)), ZZ), c.zz), H);
  *l0 = fp2_sub(fp2_mul(r, c.xz), fp2_mul(c.y2z, Z3));
  *l1 = fp2_mul(r, c.zzz_xn);
  *l3 = fp2_mul(Z3, c.zzz_yp);
  t.x = X3;
  t.y = Y3;
  t.z = Z3;
}

#ifndef BGV_MILLER_LOOP_ATTR
#define BGV_MILLER_LOOP_ATTR BGV_NOINLINE
#endif

// The line (l0 + l1 w^2 + l3 w^3) as an Fp12 value (the first step's f = 1 * line).
BGV_HD fp12_t fp12_from_line(const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
  return fp12_t{fp6_t{l0, l1, fp2_zero()}, fp6_t{fp2_zero(), l3, fp2_zero()}};
}

// ---------------------------------------------------------------------------
// The same Miller loop on lazy values (bls_lazy.h): the line formulas and the Fp12
// steps compute the same field elements as miller_dbl / miller_add_jq /
// fp12_sqr / fp12_mul_line, with the additions and subtractions left unreduced and the
// bounds checked at compile time.  T and f are brought back to < 2p once per step.
// ---------------------------------------------------------------------------
struct lz_tpt {
  lz2r x, y, z;
};
typedef lz12<LMASK, 2> lzf12;

struct lz_mp {
  lzr xn, yp, zp3;
};
struct lz_jq {
  lz2r qx, qy, qz, zz, xz, y2z, zzz_xn, zzz_yp;
};

// doubling step: lines of miller_dbl (E = 3A, F = E^2 = 9 A^2, E X = 3 A X)
BGV_MILLER_ATTR void lz_miller_dbl_lines(lz_tpt& t, const lz_mp& P, lz2r* l0, lz2r* l1, lz2r* l3) {
  const lz2r A = lz2_sqr(t.x);
  const lz2r B = lz2_sqr(t.y);
  const lz2r C = lz2_sqr(B);
  const lz2r ZZ = lz2_sqr(t.z);
  const auto D = lz2_norm(lz2_dbl(lz2_sub(lz2_sqr(lz2_norm(lz2_add(t.x, B))), lz2_add(A, C))));
  *l0 = lz2_mul_fp(lz2_sub(lz2_mulk<3>(lz2_mul(A, t.x)), lz2_dbl(B)), P.zp3);
  *l1 = lz2_mul_fp(lz2_mulk<3>(lz2_mul(A, ZZ)), P.xn);
  const auto X3 = lz2_sub(lz2_mulk<9>(lz2_sqr(A)), lz2_dbl(D));
  const auto Y3 = lz2_sub(lz2_mulk<3>(lz2_mul(A, lz2_norm(lz2_sub(D, X3)))), lz2_mulk<8>(C));
  const auto Z3 = lz2_sub(lz2_sqr(lz2_norm(lz2_add(t.y, t.z))), lz2_add(B, ZZ));
  *l3 = lz2_mul_fp(lz2_mul(lz2_wnorm(Z3), ZZ), P.yp);
  t.x = lz2_red(X3);
  t.y = lz2_red(Y3);
  t.z = lz2_red(Z3);
}

BGV_MILLER_ATTR lzf12 lz_miller_dbl_first(lz_tpt& t, const lz_mp& P) {
  lz2r l0, l1, l3;
  lz_miller_dbl_lines(t, P, &l0, &l1, &l3);
  const lz2r z = lz2r{lz_in(fp_zero()), lz_in(fp_zero())};
  return lzf12{lz6<LMASK, 2>{l0, l1, z}, lz6<LMASK, 2>{z, l3, z}};
}

// f^2 first: while it is computed only f is live (T and the P constants wait in their
// registers or spill slots untouched), and the line computation then runs beside f^2 alone
// (k_miller 11.2 vs 11.6 ms per 64,512 sets, profiles/r02s3/sqr_first_ab/)
BGV_MILLER_ATTR lzf12 lz_miller_dbl_step(const lzf12& f, lz_tpt& t, const lz_mp& P) {
  const lzf12 f2 = lz12_red(lz12_sqr(f));
  lz2r l0, l1, l3;
  lz_miller_dbl_lines(t, P, &l0, &l1, &l3);
  return lz12_red(lz12_mul_line(f2, l0, l1, l3));
}

// addition step with the Jacobian-Q constants (miller_add_jq; J = 4 H HH, V = 4 U1 HH)
BGV_MILLER_ATTR lzf12 lz_miller_add_step(const lzf12& f, lz_tpt& t, const lz_jq& c) {
  const lz2r ZZ = lz2_sqr(t.z);
  const auto U1 = lz2_mul(t.x, c.zz);
  const auto U2 = lz2_mul(c.qx, ZZ);
  const auto S1 = lz2_mul(t.y, lz2_mul(c.zz, c.qz));
  const auto S2 = lz2_mul(c.qy, lz2_mul(t.z, ZZ));
  const auto H = lz2_norm(lz2_sub(U2, U1));
  const lz2r HH = lz2_sqr(H);
  const auto J = lz2_mulk<4>(lz2_mul(H, HH));
  const lz2r r = lz2_red(lz2_dbl(lz2_sub(S2, S1)));
  const auto V = lz2_mulk<4>(lz2_mul(U1, HH));
  const auto X3 = lz2_norm(lz2_sub(lz2_sqr(r), lz2_add(J, lz2_dbl(V))));
  const auto Y3 = lz2_sub(lz2_mul(r, lz2_norm(lz2_sub(V, X3))), lz2_dbl(lz2_mul(S1, lz2_norm(J))));
  const auto Z3 = lz2_mul(lz2_wnorm(lz2_sub(lz2_sqr(lz2_norm(lz2_add(t.z, c.qz))), lz2_add(ZZ, c.zz))), H);
  const auto l0 = lz2_norm(lz2_sub(lz2_mul(r, c.xz), lz2_mul(c.y2z, Z3)));
  const lz2r l1 = lz2_red(lz2_mul(r, c.zzz_xn));
  const lz2r l3 = lz2_red(lz2_mul(Z3, c.zzz_yp));
  t.x = lz2_red(X3);
  t.y = lz2_red(Y3);
  t.z = lz2_red(Z3);
  return lz12_red(lz12_mul_line(f, l0, l1, l3));
}

// f_{|x|,Q}(P) for ONE pair (conjugated for x < 0): P and Q Jacobian (Z != 0).
// The per-set Miller loop of the blst batch equation (maybeBatch.ts:18-25 ->
// verifyMultipleAggregateSignatures): e(r_i pk_i, H(m_i)); the signature side
// e(-G1, sum r_i sig_i) is one team loop per device group (bls_team.h).
// P and Q are read from memory: the Jacobian-Q constants of the 5 addition steps (16 Fp,
// 224 VGPRs) are recomputed there from Q and P (~19 products per step) instead of staying
// live across the 63 doubling steps, where the registers hold f, T and the step's
// temporaries.  The opaque index keeps the compiler from hoisting the loads.
BGV_MILLER_LOOP_ATTR fp12_t miller_loop1m(const g1_jac* pm, const g2_jac* qm) {
  const lz_mp P = [&] {
    const miller_p P0 = miller_p_make(pm[0]);
    return lz_mp{lz_in(P0.xn), lz_in(P0.yp), lz_in(P0.zp3)};
  }();
  lz_tpt t = {lz2_in(qm[0].x), lz2_in(qm[0].y), lz2_in(qm[0].z)};
  const uint64_t X = BGV_X_ABS;
  lzf12 f = lz_miller_dbl_first(t, P);
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if ((X >> (i + 1)) & 1) {
      const int o = bgv_opaque0();
      const miller_p P0 = miller_p_make(pm[o]);
      const miller_jq c0 = miller_jq_make(qm[o], P0);
      const lz_jq c = {lz2_in(c0.q.x), lz2_in(c0.q.y), lz2_in(c0.q.z),      lz2_in(c0.zz),
                       lz2_in(c0.xz),  lz2_in(c0.y2z), lz2_in(c0.zzz_xn), lz2_in(c0.zzz_yp)};
      f = lz_miller_add_step(f, t, c);
    }
    f = lz_miller_dbl_step(f, t, P);
  }
  return fp12_conj(lz12_out(f));
}
BGV_HD fp12_t miller_loop1(const g1_jac& p, const g2_jac& q) { return miller_loop1m(&p, &q); }

// ---------------------------------------------------------------------------
// The same Miller loop split in two phases (the bulk verify path: k_lines, k_facc).
//   k_lines  walks the twist point T over the loop and emits each step's line WITHOUT the G1
//            factors (they are the only place P enters):  l0 = L0 Z_P^3,  l1 = L1 (-X_P Z_P),
//            l3 = L3 Y_P, with (L0, L1, L3) below.  Lines depend on Q only, so a signing root
//            shared by many sets is walked once (hash_to_G2 once per root, bgv_dslot.hsrc).
//   k_facc   keeps only f and P: per step f <- f^2 * (L scaled by P).
// The scaled lines are the same field elements as lz_miller_dbl_lines / miller_add_jq's, so
// f is the same field element as miller_loop1m's (bit-identical after canonicalisation).
// Line record: 68 steps (the first doubling, then per bit 61..0 an addition where the next
// bit of |x| is set and a doubling) x (L0, L1, L3) = 6 Fp = 84 u32 limbs.
// ---------------------------------------------------------------------------
#define BGV_MILLER_STEPS 68
#define BGV_LINE_WORDS (6 * NL)
#define BGV_LINE_QUADS (BGV_LINE_WORDS / 4)

template <class A, class B, class C>
struct lz_pline_t {
  A L0;
  B L1;
  C L3;
};

// doubling step: L0 = 3 X^3 - 2 Y^2, L1 = 3 X^2 Z^2, L3 = Z3 Z^2 (E = 3A as in lz_miller_dbl_lines)
BGV_MILLER_ATTR auto lz_pline_dbl(lz_tpt& t) {
  const lz2r A = lz2_sqr(t.x);
  const lz2r B = lz2_sqr(t.y);
  const lz2r C = lz2_sqr(B);
  const lz2r ZZ = lz2_sqr(t.z);
  const auto D = lz2_norm(lz2_dbl(lz2_sub(lz2_sqr(lz2_norm(lz2_add(t.x, B))), lz2_add(A, C))));
  const auto L0 = lz2_norm(lz2_sub(lz2_mulk<3>(lz2_mul(A, t.x)), lz2_dbl(B)));
  const auto L1 = lz2_norm(lz2_mulk<3>(lz2_mul(A, ZZ)));
  const auto X3 = lz2_sub(lz2_mulk<9>(lz2_sqr(A)), lz2_dbl(D));
  const auto Y3 = lz2_sub(lz2_mulk<3>(lz2_mul(A, lz2_norm(lz2_sub(D, X3)))), lz2_mulk<8>(C));
  const auto Z3 = lz2_sub(lz2_sqr(lz2_norm(lz2_add(t.y, t.z))), lz2_add(B, ZZ));
  const auto L3 = lz2_norm(lz2_mul(lz2_wnorm(Z3), ZZ));
  t.x = lz2_red(X3);
  t.y = lz2_red(Y3);
  t.z = lz2_red(Z3);
  return lz_pline_t<std::decay_t<decltype(L0)>, std::decay_t<decltype(L1)>, std::decay_t<decltype(L3)>>{L0, L1, L3};
}

// addition step T + Q, Q = (X2 : Y2 : Z2) Jacobian (miller_add_jq without the P factors):
// L0 = r X2 Z2 - Y2 Z3, L1 = r Z2^3, L3 = Z3 Z2^3
BGV_MILLER_ATTR auto lz_pline_add(lz_tpt& t, const lz2r& qx, const lz2r& qy, const lz2r& qz) {
  const lz2r zz = lz2_sqr(qz);
  const auto zzz = lz2_norm(lz2_mul(zz, qz));
  const auto xz = lz2_norm(lz2_mul(qx, qz));
  const lz2r ZZ = lz2_sqr(t.z);
  const auto U1 = lz2_mul(t.x, zz);
  const auto U2 = lz2_mul(qx, ZZ);
  const auto S1 = lz2_mul(t.y, zzz);
  const auto S2 = lz2_mul(qy, lz2_mul(t.z, ZZ));
  const auto H = lz2_norm(lz2_sub(U2, U1));
  const lz2r HH = lz2_sqr(H);
  const auto J = lz2_mulk<4>(lz2_mul(H, HH));
  const lz2r r = lz2_red(lz2_dbl(lz2_sub(S2, S1)));
  const auto V = lz2_mulk<4>(lz2_mul(U1, HH));
  const auto X3 = lz2_norm(lz2_sub(lz2_sqr(r), lz2_add(J, lz2_dbl(V))));
  const auto Y3 = lz2_sub(lz2_mul(r, lz2_norm(lz2_sub(V, X3))), lz2_dbl(lz2_mul(S1, lz2_norm(J))));
  const auto Z3 = lz2_mul(lz2_wnorm(lz2_sub(lz2_sqr(lz2_norm(lz2_add(t.z, qz))), lz2_add(ZZ, zz))), H);
  const auto L0 = lz2_norm(lz2_sub(lz2_mul(r, xz), lz2_mul(qy, Z3)));
  const auto L1 = lz2_norm(lz2_mul(r, zzz));
  const auto L3 = lz2_norm(lz2_mul(Z3, zzz));
  t.x = lz2_red(X3);
  t.y = lz2_red(Y3);
  t.z = lz2_red(Z3);
  return lz_pline_t<std::decay_t<decltype(L0)>, std::decay_t<decltype(L1)>, std::decay_t<decltype(L3)>>{L0, L1, L3};
}

// Round 6: the bulk walk (k_lines) in homogeneous projective coordinates, x = X/Z, y = Y/Z.
// Doubling (a = 0, b' = 4(1 + i); Costello-Lange-Naehrig, all coordinates times 4): B = Y^2,
// C = Z^2, E = 3 b' C, F = 3E, H = (Y + Z)^2 - B - C = 2YZ,
//   X3 = 2XY (B - F), Y3 = (B + F)^2 - 12 E^2, Z3 = 4 B H,
// and the tangent scaled by 2YZ: H yP - 3X^2 xP + (B - E), i.e. L0 = B - E, L1 = 3X^2, L3 = H in
// the records' convention (l = L0 - L1 xP + L3 yP, scaled by P as before): 3 products + 6
// squarings against the Jacobian step's 4 + 7.  Addition T + Q (Q projective; add-1998-cmo-2):
// u = Y2 Z1 - Y1 Z2, v = X2 Z1 - X1 Z2, X3 = v A, Y3 = u (R - A) - v^3 Y1 Z2, Z3 = v^3 Z1 Z2
// (R = v^2 X1 Z2, A = u^2 Z1 Z2 - v^3 - 2R), the chord through Q scaled by v Z2:
// L0 = u X2 - v Y2, L1 = u Z2, L3 = v Z2.  Other representatives of the same lines (Fp2
// factors the final exponentiation removes): the same pairing values as the Jacobian walk
// (tests/test_pairing_golden.py, and on the device tests/test_gpu_pairing.py).
BGV_MILLER_ATTR auto lz_pline_dbl_p(lz_tpt& t) {
  const lz2r B = lz2_sqr(t.y);
  const lz2r C = lz2_sqr(t.z);
  const lz2r XX = lz2_sqr(t.x);
  const lz2r E = lz2_red(lz2_mulk<12>(lz2_norm(lz2_mul_xi(C))));  // 3 b' C = 12 (1 + i) C
  const auto F = lz2_mulk<3>(E);
  const auto H = lz2_norm(lz2_sub(lz2_sqr(lz2_norm(lz2_add(t.y, t.z))), lz2_add(B, C)));
  const auto XY = lz2_mul(t.x, t.y);
  const auto X3 = lz2_mul(lz2_wnorm(lz2_dbl(XY)), lz2_wnorm(lz2_norm(lz2_sub(B, F))));
  const auto Y3 = lz2_sub(lz2_sqr(lz2_norm(lz2_add(B, F))), lz2_mulk<12>(lz2_sqr(E)));
  const auto Z3 = lz2_mulk<4>(lz2_mul(B, H));
  const auto L0 = lz2_norm(lz2_sub(B, E));
  const auto L1 = lz2_norm(lz2_mulk<3>(XX));
  const auto L3 = H;
  t.x = lz2_red(X3);
  t.y = lz2_red(Y3);
  t.z = lz2_red(Z3);
  return lz_pline_t<std::decay_t<decltype(L0)>, std::decay_t<decltype(L1)>, std::decay_t<decltype(L3)>>{L0, L1, L3};
}
BGV_MILLER_ATTR auto lz_pline_add_p(lz_tpt& t, const lz2r& qx, const lz2r& qy, const lz2r& qz) {
  const auto Y1Z2 = lz2_mul(t.y, qz);
  const auto X1Z2 = lz2_mul(t.x, qz);
  const auto Z1Z2 = lz2_mul(t.z, qz);
  const auto u = lz2_norm(lz2_sub(lz2_mul(qy, t.z), Y1Z2));
  const auto v = lz2_norm(lz2_sub(lz2_mul(qx, t.z), X1Z2));
  const lz2r uu = lz2_sqr(u);
  const lz2r vv = lz2_sqr(v);
  const auto vvv = lz2_mul(v, vv);
  const auto R = lz2_mul(vv, X1Z2);
  const auto A = lz2_norm(lz2_sub(lz2_mul(uu, Z1Z2), lz2_add(vvv, lz2_dbl(R))));
  const auto X3 = lz2_mul(v, A);
  const auto Y3 = lz2_sub(lz2_mul(u, lz2_wnorm(lz2_norm(lz2_sub(R, A)))), lz2_mul(vvv, Y1Z2));
  const auto Z3 = lz2_mul(vvv, Z1Z2);
  const auto L0 = lz2_norm(lz2_sub(lz2_mul(u, qx), lz2_mul(v, qy)));
  const auto L1 = lz2_norm(lz2_mul(u, qz));
  const auto L3 = lz2_norm(lz2_mul(v, qz));
  t.x = lz2_red(X3);
  t.y = lz2_red(Y3);
  t.z = lz2_red(Z3);
  return lz_pline_t<std::decay_t<decltype(L0)>, std::decay_t<decltype(L1)>, std::decay_t<decltype(L3)>>{L0, L1, L3};
}
// Jacobian Q (x = X/Z^2, y = Y/Z^3) as projective: (X Z, Y, Z^3)
BGV_HD lz_tpt lz_tpt_proj(const g2_jac& q) {
  const lz2r z = lz2_in(q.z);
  return lz_tpt{lz2_red(lz2_mul(lz2_in(q.x), z)), lz2_in(q.y), lz2_red(lz2_mul(lz2_sqr(z), z))};
}

// the record types the two phases agree on
#if defined(BGV_LINES_JACOBIAN)  // A/B: round 5's Jacobian walk
typedef decltype(lz_pline_dbl(*(lz_tpt*)nullptr)) lz_pline_d;
typedef decltype(lz_pline_add(*(lz_tpt*)nullptr, lz2r{}, lz2r{}, lz2r{})) lz_pline_a;
#else
typedef decltype(lz_pline_dbl_p(*(lz_tpt*)nullptr)) lz_pline_d;
typedef decltype(lz_pline_add_p(*(lz_tpt*)nullptr, lz2r{}, lz2r{}, lz2r{})) lz_pline_a;
#endif

// the line of a record scaled by P (6 products), as an Fp12 factor's three coefficients
template <class Lp>
BGV_HD void lz_pline_scale(const Lp& L, const lz_mp& P, lz2r* l0, lz2r* l1, lz2r* l3) {
  *l0 = lz2_mul_fp(L.L0, P.zp3);
  *l1 = lz2_mul_fp(L.L1, P.xn);
  *l3 = lz2_mul_fp(L.L3, P.yp);
}

// k_facc's steps: the first doubling (f = its line), an addition (f * line), a doubling (f^2 * line)
template <class Lp>
BGV_HD lzf12 lz_facc_first(const Lp& L, const lz_mp& P) {
  lz2r l0, l1, l3;
  lz_pline_scale(L, P, &l0, &l1, &l3);
  const lz2r z = lz2r{lz_in(fp_zero()), lz_in(fp_zero())};
  return lzf12{lz6<LMASK, 2>{l0, l1, z}, lz6<LMASK, 2>{z, l3, z}};
}
template <class Lp>
BGV_HD lzf12 lz_facc_add(const lzf12& f, const Lp& L, const lz_mp& P) {
  lz2r l0, l1, l3;
  lz_pline_scale(L, P, &l0, &l1, &l3);
  return lz12_red(lz12_mul_line(f, l0, l1, l3));
}
// scaling with P's constants fetched at the point of use (k_facc keeps them in LDS); z is an
// opaque 0 the fetches depend on, so the compiler cannot hoist them ahead of f^2
template <class Lp, class PF>
BGV_HD void lz_pline_scale_f(const Lp& L, PF pget, uint32_t z, lz2r* l0, lz2r* l1, lz2r* l3) {
  *l0 = lz2_mul_fp(L.L0, pget(2, z));
  *l1 = lz2_mul_fp(L.L1, pget(0, z));
  *l3 = lz2_mul_fp(L.L3, pget(1, z));
}

// A word that is always 0 but depends on every coefficient of f: an index built from it keeps
// the compiler from issuing a step's record loads before f^2 exists (hoisted, the 84 loaded
// words stay live across the whole squaring and push f's temporaries into scratch).
BGV_HD uint32_t lz12_after(const lzf12& f) {
  uint32_t z = 0;
  const lz2r* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  BGV_UNROLL for (int i = 0; i < 6; ++i) z ^= c[i]->c0.v[0] ^ c[i]->c1.v[0];
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("v_mov_b32 %0, 0" : "=v"(z) : "v"(z));
#else
  asm volatile("" : "+r"(z));
  z = 0;
#endif
  return z;
}
template <class Load>
BGV_HD lzf12 lz_facc_dbl_load(const lzf12& f, int k, Load load, const lz_mp& P) {
  const lzf12 f2 = lz12_red(lz12_sqr(f));
  lz_pline_d L;
  load(k + (int)lz12_after(f2), &L);
  lz2r l0, l1, l3;
  lz_pline_scale(L, P, &l0, &l1, &l3);
  return lz12_red(lz12_mul_line(f2, l0, l1, l3));
}

// bit i + 1 of |x| is set: an addition step precedes doubling step i (i = 61..0)
BGV_HD bool miller_add_at(int i) { return (BGV_X_ABS >> (i + 1)) & 1; }

// The line records of one twist point in loop order (k_lines' walk; also the host reference).
// Q is read from memory at the 5 additions (an opaque index keeps the compiler from hoisting
// the loads), so the 63 doublings keep only T and their temporaries live.
template <class Emit>
BGV_HD void miller_lines_walk(const g2_jac* qm, Emit emit) {
#if defined(BGV_LINES_JACOBIAN)
  lz_tpt t = {lz2_in(qm[0].x), lz2_in(qm[0].y), lz2_in(qm[0].z)};
  int k = 0;
  emit(k++, lz_pline_dbl(t));
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if (miller_add_at(i)) {
      const g2_jac& q = qm[bgv_opaque0()];
      emit(k++, lz_pline_add(t, lz2_in(q.x), lz2_in(q.y), lz2_in(q.z)));
    }
    emit(k++, lz_pline_dbl(t));
  }
#else
  lz_tpt t = lz_tpt_proj(qm[0]);
  int k = 0;
  emit(k++, lz_pline_dbl_p(t));
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if (miller_add_at(i)) {
      const lz_tpt q = lz_tpt_proj(qm[bgv_opaque0()]);  // Q again from memory: not live across the doublings
      emit(k++, lz_pline_add_p(t, q.x, q.y, q.z));
    }
    emit(k++, lz_pline_dbl_p(t));
  }
#endif
}

// k_facc's walk with the records and P's constants in LDS: load(k, rec) fills record k,
// pget(j) returns P's constant j (0 xn = -X Z, 1 yp = Y, 2 zp3 = Z^3).  The record of a
// doubling is read after f^2 (lz12_after), when only f^2 is live.
template <class Load, class PF>
BGV_HD fp12_t miller_facc_walk_staged(Load load, PF pget) {
  lz2r l0, l1, l3;
  int k = 0;
  lz_pline_d d;
  load(k++, 0u, &d);
  lz_pline_scale_f(d, pget, 0u, &l0, &l1, &l3);
  const lz2r z = lz2r{lz_in(fp_zero()), lz_in(fp_zero())};
  lzf12 f = lzf12{lz6<LMASK, 2>{l0, l1, z}, lz6<LMASK, 2>{z, l3, z}};
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if (miller_add_at(i)) {
      const uint32_t za = lz12_after(f);
      lz_pline_a a;
      load(k++, za, &a);
      lz_pline_scale_f(a, pget, za, &l0, &l1, &l3);
      f = lz12_red(lz12_mul_line(f, l0, l1, l3));
    }
    const lzf12 f2 = lz12_red(lz12_sqr(f));
    const uint32_t zd = lz12_after(f2);
    load(k++, zd, &d);
    lz_pline_scale_f(d, pget, zd, &l0, &l1, &l3);
    f = lz12_red(lz12_mul_line(f2, l0, l1, l3));
  }
  return fp12_conj(lz12_out(f));
}

// k_facc's walk over one pair's records (load(k, rec) fills record k); returns f, conjugated
template <class Load>
BGV_HD fp12_t miller_facc_walk(const g1_jac& p, Load load) {
  const miller_p P0 = miller_p_make(p);
  const lz_mp P = {lz_in(P0.xn), lz_in(P0.yp), lz_in(P0.zp3)};
  int k = 0;
  lz_pline_d d;
  load(k++, &d);
  lzf12 f = lz_facc_first(d, P);
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if (miller_add_at(i)) {
      lz_pline_a a;
      load(k++, &a);
      f = lz_facc_add(f, a, P);
    }
    f = lz_facc_dbl_load(f, k++, load, P);
  }
  return fp12_conj(lz12_out(f));
}

// a^|x| in the cyclotomic subgroup, conjugated: a^x (x < 0)
BGV_NOINLINE fp12_t cyclotomic_pow_x(const fp12_t& a) {
  const uint64_t X = BGV_X_ABS;
  fp12_t r = a;
  BGV_NO_UNROLL for (int i = 62; i >= 0; --i) {
    r = fp12_cyclotomic_sqr(r);
    if ((X >> i) & 1) r = fp12_mul(r, a);
  }
  return fp12_conj(r);
}

// f^(3 (p^12 - 1) / r) using 3 (p^4 - p^2 + 1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3
BGV_NOINLINE fp12_t final_exp(const fp12_t& f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  fp12_t t = fp12_mul(fp12_conj(f), fp12_inv(f));
  t = fp12_mul(fp12_frob2(t), t);
  // hard part
  fp12_t a = fp12_mul(cyclotomic_pow_x(t), fp12_conj(t));  // t^(x-1)
  a = fp12_mul(cyclotomic_pow_x(a), fp12_conj(a));         // t^((x-1)^2)
  a = fp12_mul(cyclotomic_pow_x(a), fp12_frob(a));         // ^(x+p)
  fp12_t b = cyclotomic_pow_x(cyclotomic_pow_x(a));        // a^(x^2)
  b = fp12_mul(fp12_mul(b, fp12_frob2(a)), fp12_conj(a));  // a^(x^2 + p^2 - 1)
  fp12_t t3 = fp12_mul(fp12_cyclotomic_sqr(t), t);         // t^3
  return fp12_mul(b, t3);
}
