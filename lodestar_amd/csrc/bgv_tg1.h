// Team G1 scalar multiplication for the latency path: r_i * pk_i from the generated point
// programs of bgv_tg1_prog.h (tools/gen_tg1.py; the round model of bgv_tmiller.h), so the
// pubkey task of k_prep_wide no longer runs its 64-bit multiplication on one lane (~670
// chained products) while the other tasks' chains run as rounds.
//
// The schedule restates bls_curve.h jac_mul_glv<fp_t> (r = lo32 + hi32 x^2, 2-bit windows,
// E = (beta X, -Y, Z) = [x^2] on G1) exactly as bgv_tcurve.h tc_mul_glv does for G2, in
// homogeneous projective coordinates with Jacobian in and out: the same point as the one-lane
// formulas, another representative.  Both halves' prefixes stay below 2^32 < x^2, so the
// accumulator never meets an entry or its negative once finite: the generic additions are
// exact; P must be finite and in G1 (a cached, aggregated or validated key).
#pragma once
#include "bgv_tmiller.h"
#include "bgv_tg1_prog.h"

// r P: P in bank 1 on entry, the result in bank 4 (both Jacobian).  Tables: P, 2P, 3P in
// banks 1-3 and E of them in banks 6-8; banks 4 / 5 the accumulator, bank 0 the entry added.
template <class E>
BGV_HD void tg1_mul_glv(E& e, uint64_t k) {
  const uint32_t a = (uint32_t)k, b = (uint32_t)(k >> 32);
  e.run(TG1_J2P1_4);
  e.copy(1, 4);
  e.copy(0, 1);        // P
  e.run(TG1_PDBL45);   // 2P
  e.copy(2, 5);
  e.run(TG1_PADD123);  // 3P
  e.copy(9, 2);
  e.run(TG1_ENDO12);   // E(P)
  e.copy(6, 2);
  e.copy(1, 9);
  e.run(TG1_ENDO12);   // E(2P)
  e.copy(7, 2);
  e.copy(1, 3);
  e.run(TG1_ENDO12);   // E(3P)
  e.copy(8, 2);
  e.copy(1, 0);
  e.copy(2, 9);
  bool inf = true;
  for (int i = 30; i >= 0; i -= 2) {
    e.run(TG1_PDBL45);
    e.run(TG1_PDBL54);
    const int da = (int)((a >> i) & 3u);
    e.copy(0, da ? da : 1);
    e.run(TG1_PADD405);
    e.copy(4, da == 0 ? 4 : (inf ? 0 : 5));
    inf = inf && da == 0;
    const int db = (int)((b >> i) & 3u);
    e.copy(0, db ? 5 + db : 6);
    e.run(TG1_PADD405);
    e.copy(4, db == 0 ? 4 : (inf ? 0 : 5));
    inf = inf && db == 0;
  }
  e.copy(3, 4);
  e.run(TG1_P2J31);
  e.copy(4, 1);
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host emulation (tests): programs lane by lane, bank moves as plain copies.
struct tg1_host_engine {
  const uint8_t* tab;
  fp_t* S;
  void run(int off) { tmp_run_host(tab, off, S); }
  void copy(int dst, int src) {
    if (dst == src) return;
    for (int i = 0; i < 3; ++i) S[TG1_BANK(dst) + i] = S[TG1_BANK(src) + i];
  }
};

inline g1_jac tg1_mul_glv_host(const g1_jac& p, uint64_t k) {
  static const uint8_t tab[TG1_TABLE_BYTES] = TG1_TABLE_INIT;
  static fp_t S[TG1_NSLOT];
  for (int i = 0; i < TG1_NSLOT; ++i) S[i] = fp_zero();
  S[TG1_S_ONE] = fp_one();
  S[TG1_S_BETA] = fp_t{BGV_BETA_MX2};
  S[TG1_BANK(1)] = p.x;
  S[TG1_BANK(1) + 1] = p.y;
  S[TG1_BANK(1) + 2] = p.z;
  tg1_host_engine e{tab, S};
  tg1_mul_glv(e, k);
  return g1_jac{S[TG1_BANK(4)], S[TG1_BANK(4) + 1], S[TG1_BANK(4) + 2]};
}
#endif
