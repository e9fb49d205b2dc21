// Team G2 scalar multiplications for the latency path: the cofactor clearing of hash_to_G2
// and r_i * sig_i on a team of 16 lanes (one set per team), from the generated point
// programs of bgv_tcurve_prog.h (tools/gen_tcurve.py; the round model of bgv_tmiller.h).
//
// The chains run in homogeneous projective coordinates (tools/gen_tcurve.py): a doubling is
// 2 rounds and an addition 3 (Jacobian: 3 and 5), against ~16 and ~43 chained products on one
// lane.  Every schedule converts its input banks from Jacobian and its result back (j2p /
// p2j programs), so callers hand in and take out Jacobian points as before: the same points
// as bls_curve.h's formulas give, other representatives.  The schedules below restate bls_curve.h
// step by step (g2_clear_cofactor, jac_mul_u64) over point "banks" of six LDS slots; the
// engine E supplies the program runs and the bank moves, so the same schedule runs on the
// device (bgv_k_prep.hip) and in the host emulation (tests/native/hostsim.cpp).
//
// The additions are the generic-case formulas.  tc_clear_cofactor flags an addition whose
// inputs share x or include infinity (v^2 or Z1 Z2 zero) and the caller then recomputes
// with the complete one-lane formulas; for hash outputs this never happens in practice.
// In tc_mul_u64 the only exceptional addition is the first (accumulator at infinity), which
// the schedule handles by selecting the table entry instead.
#pragma once
#include "bgv_tmiller.h"
#include "bgv_tcurve_prog.h"

// the addition programs' exceptional-case witnesses: v^2 and Z1 Z2 (tools/gen_tcurve.py)
#define TC_CHK_A TCP_S_VV
#define TC_CHK_B TCP_S_ZZ

// The isogeny programs' constant slots: x_num[4], x_den[2], y_num[4], y_den[3] (Fp2, bls_hash.h
// iso_map_g2_jac) as TC_ISO_NCONST Fp values from TCP_S_ISO on; every engine's slots hold them.
#define TC_ISO_NCONST 26
BGV_HD fp_t tc_iso_const(int i) {
  const fp2_t xn[4] = BGV_ISO_XNUM, xd[2] = BGV_ISO_XDEN, yn[4] = BGV_ISO_YNUM, yd[3] = BGV_ISO_YDEN;
  const int k = i >> 1;
  const fp2_t& v = k < 4 ? xn[k] : (k < 6 ? xd[k - 4] : (k < 10 ? yn[k - 6] : yd[k - 10]));
  return (i & 1) ? v.c1 : v.c0;
}

// the projective point in bank b -> Jacobian in bank 1 (returns 1)
template <class E>
BGV_HD int tc_to_jac(E& e, int b) {
  e.copy(3, b);
  e.run(TCP_P2J31);
  return 1;
}

// [|x|]P, projective: base in bank 0, accumulator (= P) in bank 4 on entry; returns the
// result's bank
template <class E>
BGV_HD int tc_mul_x_abs(E& e) {
  int acc = 4;
  for (int i = 62; i >= 0; --i) {
    e.run(acc == 4 ? TCP_PDBL45 : TCP_PDBL54);
    acc = 9 - acc;
    if ((BGV_X_ABS >> i) & 1) {
      e.run(acc == 4 ? TCP_PADD405 : TCP_PADD504);
      e.check_add();
      acc = 9 - acc;
    }
  }
  return acc;
}

// RFC 9380 G.4 (bls_curve.h g2_clear_cofactor) of iso(q0) + iso(q1): the SSWU points q0 in
// bank 1, q1 in bank 2 on entry (on E2', Jacobian), the result in bank 3 (Jacobian).  Storage
// banks: 6 = P, 7 = t1, 8 = t2, 9 = t3.
template <class E>
BGV_HD void tc_clear_cofactor(E& e) {
  e.run(TCP_ISO12_45);  // the 3-isogeny of q0, q1 into projective banks 4, 5
  e.copy(1, 4);
  e.copy(2, 5);
  e.run(TCP_PADD123);  // P = q0 + q1
  e.check_add();
  e.copy(6, 3);
  e.copy(0, 3);
  e.copy(4, 3);
  int a = tc_mul_x_abs(e);  // t1 = [x]P = -[|x|]P
  e.neg_y(a);
  e.copy(7, a);
  e.copy(1, 6);  // t2 = psi(P)
  e.run(TCP_PSI12);
  e.copy(8, 2);
  e.copy(4, 6);  // t3 = psi2(2P)
  e.run(TCP_PDBL45);
  e.copy(1, 5);
  e.run(TCP_PSI2_12);
  e.copy(9, 2);
  e.copy(1, 9);  // t3 = t3 - t2
  e.copy(2, 8);
  e.neg_y(2);
  e.run(TCP_PADD123);
  e.check_add();
  e.copy(9, 3);
  e.copy(1, 7);  // t2 = [x](t1 + t2)
  e.copy(2, 8);
  e.run(TCP_PADD123);
  e.check_add();
  e.copy(0, 3);
  e.copy(4, 3);
  a = tc_mul_x_abs(e);
  e.neg_y(a);
  e.copy(8, a);
  e.copy(1, 9);  // t3 = t3 + t2
  e.copy(2, 8);
  e.run(TCP_PADD123);
  e.check_add();
  e.copy(9, 3);
  e.copy(1, 9);  // t3 = t3 - t1
  e.copy(2, 7);
  e.neg_y(2);
  e.run(TCP_PADD123);
  e.check_add();
  e.copy(9, 3);
  e.copy(1, 9);  // t3 - P
  e.copy(2, 6);
  e.neg_y(2);
  e.run(TCP_PADD123);
  e.check_add();
  tc_to_jac(e, 3);
  e.copy(3, 1);
}

// [k]P for the team's 64-bit k (bls_curve.h jac_mul_u64: 2-bit fixed window over the table
// P, 2P, 3P): P in bank 1 on entry, the result in bank 4 (both Jacobian).  Every window runs the same
// programs on every team (lane-uniform control flow); the per-team digit only picks bank
// sources: table entry d -> bank 0, and the new accumulator from bank 4 (d = 0), bank 5
// (acc + entry) or bank 0 (accumulator still at infinity).
template <class E>
BGV_HD void tc_mul_u64(E& e, uint64_t k) {
  e.run(TCP_J2P12_45);
  e.copy(1, 4);
  e.run(TCP_PDBL45);
  e.copy(2, 5);        // 2P
  e.run(TCP_PADD123);  // 3P
  bool inf = true;
  for (int i = 62; i >= 0; i -= 2) {
    e.run(TCP_PDBL45);
    e.run(TCP_PDBL54);
    const int d = (int)((k >> i) & 3u);
    e.copy(0, d ? d : 1);
    e.run(TCP_PADD405);
    e.copy(4, d == 0 ? 4 : (inf ? 0 : 5));
    inf = inf && d == 0;
  }
  e.copy(4, tc_to_jac(e, 4));
}

// r P for the randomizer r = lo32(k) + hi32(k) x^2 (bls_curve.h jac_mul_glv) with 2-bit
// windows: P in bank 1 on entry, the result in bank 4 (both Jacobian).  Tables: P, 2P, 3P in banks 1-3 and
// psi^2 of them (= [x^2] times, P in G2) in banks 6-8.  Per window: two doublings, then the
// a-digit's and the b-digit's entries added through bank 0 (the per-team digit picks the
// source bank), the accumulator taking the entry itself while it is still at infinity.
// Both halves' prefixes are < 2^32 < x^2, so the accumulator never equals an entry or its
// negative once it is finite: the generic addition programs are exact here.
template <class E>
BGV_HD void tc_mul_glv(E& e, uint64_t k) {
  const uint32_t a = (uint32_t)k, b = (uint32_t)(k >> 32);
  e.run(TCP_J2P12_45);
  e.copy(1, 4);
  e.copy(0, 1);  // P
  e.run(TCP_PDBL45);
  e.copy(2, 5);        // 2P
  e.run(TCP_PADD123);  // 3P
  e.copy(9, 2);
  e.run(TCP_PSI2_12);  // bank 1 still P
  e.copy(6, 2);
  e.copy(1, 9);
  e.run(TCP_PSI2_12);
  e.copy(7, 2);
  e.copy(1, 3);
  e.run(TCP_PSI2_12);
  e.copy(8, 2);
  e.copy(1, 0);
  e.copy(2, 9);
  bool inf = true;
  for (int i = 30; i >= 0; i -= 2) {
    e.run(TCP_PDBL45);
    e.run(TCP_PDBL54);
    const int da = (int)((a >> i) & 3u);
    e.copy(0, da ? da : 1);
    e.run(TCP_PADD405);
    e.copy(4, da == 0 ? 4 : (inf ? 0 : 5));
    inf = inf && da == 0;
    const int db = (int)((b >> i) & 3u);
    e.copy(0, db ? 5 + db : 6);
    e.run(TCP_PADD405);
    e.copy(4, db == 0 ? 4 : (inf ? 0 : 5));
    inf = inf && db == 0;
  }
  e.copy(4, tc_to_jac(e, 4));
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host emulation engine (tests): programs lane by lane, bank moves as plain copies.
struct tc_host_engine {
  const uint8_t* tab;
  fp_t* S;
  bool bad = false;
  void run(int off) { tmp_run_host(tab, off, S); }
  void copy(int dst, int src) {
    if (dst == src) return;
    for (int i = 0; i < 6; ++i) S[TCP_BANK(dst) + i] = S[TCP_BANK(src) + i];
  }
  void neg_y(int b) {
    S[TCP_BANK(b) + 2] = fp_neg(S[TCP_BANK(b) + 2]);
    S[TCP_BANK(b) + 3] = fp_neg(S[TCP_BANK(b) + 3]);
  }
  void check_add() {
    const auto z2 = [&](int s) { return fp_is_zero(S[s]) && fp_is_zero(S[s + 1]); };
    bad = bad || z2(TC_CHK_A) || z2(TC_CHK_B);
  }
};

inline void tc_host_init(fp_t* S) {
  for (int i = 0; i < TCP_NSLOT; ++i) S[i] = fp_zero();
  for (int i = 0; i < TC_ISO_NCONST; ++i) S[TCP_S_ISO + i] = tc_iso_const(i);
  const fp2_t cx = BGV_PSI_CX, cy = BGV_PSI_CY;
  S[TCP_S_ONE] = fp_one();
  S[TCP_S_PSI_CX] = cx.c0;
  S[TCP_S_PSI_CX + 1] = cx.c1;
  S[TCP_S_PSI_CY] = cy.c0;
  S[TCP_S_PSI_CY + 1] = cy.c1;
  S[TCP_S_PSI2_CX] = fp_t{BGV_PSI2_CX};
  S[TCP_S_PSI2_CY] = fp_t{BGV_PSI2_CY};
}

inline void tc_put(fp_t* S, int b, const g2_jac& p) {
  const fp_t v[6] = {p.x.c0, p.x.c1, p.y.c0, p.y.c1, p.z.c0, p.z.c1};
  for (int i = 0; i < 6; ++i) S[TCP_BANK(b) + i] = v[i];
}
inline g2_jac tc_get(const fp_t* S, int b) {
  const fp_t* v = S + TCP_BANK(b);
  return g2_jac{fp2_t{v[0], v[1]}, fp2_t{v[2], v[3]}, fp2_t{v[4], v[5]}};
}

// g2_clear_cofactor(iso(q0) + iso(q1)) of two SSWU points and [k]P through the team schedules
// (*bad: the cofactor clearing met an exceptional addition)
inline g2_jac tc_clear_cofactor_host(const g2_jac& q0, const g2_jac& q1, bool* bad) {
  static const uint8_t tab[TCP_TABLE_BYTES] = TCP_TABLE_INIT;
  static fp_t S[TCP_NSLOT];
  tc_host_init(S);
  tc_put(S, 1, q0);
  tc_put(S, 2, q1);
  tc_host_engine e{tab, S};
  tc_clear_cofactor(e);
  *bad = e.bad;
  return tc_get(S, 3);
}
inline g2_jac tc_mul_u64_host(const g2_jac& p, uint64_t k) {
  static const uint8_t tab[TCP_TABLE_BYTES] = TCP_TABLE_INIT;
  static fp_t S[TCP_NSLOT];
  tc_host_init(S);
  tc_put(S, 1, p);
  tc_host_engine e{tab, S};
  tc_mul_u64(e, k);
  return tc_get(S, 4);
}
inline g2_jac tc_mul_glv_host(const g2_jac& p, uint64_t k) {
  static const uint8_t tab[TCP_TABLE_BYTES] = TCP_TABLE_INIT;
  static fp_t S[TCP_NSLOT];
  tc_host_init(S);
  tc_put(S, 1, p);
  tc_host_engine e{tab, S};
  tc_mul_glv(e, k);
  return tc_get(S, 4);
}
#endif
