// TEST-ONLY host build of the device arithmetic (lodestar_amd/csrc/bls_*.h).
//
// The kernels' per-lane math is plain C++ in __host__ __device__ headers, so
// the exact same formulas are compiled here with g++ and exercised from
// pytest against oracle/bls12381.py on a machine without a GPU.  Nothing in
// the product links this library; the product path is the HIP build only.
#include <string.h>

#include "../../lodestar_amd/csrc/bls_hash.h"
#include "../../lodestar_amd/csrc/bls_pairing.h"
#include "../../lodestar_amd/csrc/bls_team.h"
#include "../../lodestar_amd/csrc/bgv_tmiller.h"
#include "../../lodestar_amd/csrc/bgv_tcurve.h"
#include "../../lodestar_amd/csrc/bgv_tg1.h"

static fp_t in_fp(const uint8_t* be) { return fp_to_mont(fp_from_be48(be)); }
static void out_fp(uint8_t* be, const fp_t& a) { fp_to_be48(be, fp_from_mont(a)); }
static fp2_t in_fp2(const uint8_t* be) { return fp2_t{in_fp(be), in_fp(be + 48)}; }  // (c0, c1)
static void out_fp2(uint8_t* be, const fp2_t& a) {
  out_fp(be, a.c0);
  out_fp(be + 48, a.c1);
}
static void out_fp12(uint8_t* be, const fp12_t& f) {
  const fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; ++i) out_fp2(be + 96 * i, *c[i]);
}
static fp12_t in_fp12(const uint8_t* be) {
  fp12_t f;
  fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; ++i) *c[i] = in_fp2(be + 96 * i);
  return f;
}
// G2 affine as x.c0 | x.c1 | y.c0 | y.c1 (48 B each, raw BE) -- test layout
static g2_aff in_g2(const uint8_t* be) { return g2_aff{in_fp2(be), in_fp2(be + 96)}; }
static void out_g2(uint8_t* be, const g2_aff& a) {
  out_fp2(be, a.x);
  out_fp2(be + 96, a.y);
}
static g1_aff in_g1(const uint8_t* be) { return g1_aff{in_fp(be), in_fp(be + 48)}; }
static void out_g1(uint8_t* be, const g1_aff& a) {
  out_fp(be, a.x);
  out_fp(be + 48, a.y);
}

extern "C" {
#ifdef BGV_COUNT_OPS
unsigned long long bgv_count_mul = 0, bgv_count_sqr = 0;
void hs_count_reset() { bgv_count_mul = bgv_count_sqr = 0; }
unsigned long long hs_count_mul() { return bgv_count_mul; }
unsigned long long hs_count_sqr() { return bgv_count_sqr; }
// per-lane bodies of the verify kernels (bgv_kernels.hip), for counting only
int hs_k_sig_body(const uint8_t* sig96, uint64_t r) {
  g2_aff a;
  bool inf;
  if (g2_decompress(&a, &inf, sig96) || inf) return 0;
  if (!g2_in_subgroup(jac_from_aff(a))) return 0;
  return !jac_is_inf(jac_mul_glv(jac_from_aff(a), r));  // r * sig for the group sum
}
int hs_k_hash_body(const uint8_t* msg32) { return !jac_is_inf(hash_to_g2(msg32, 32)); }
int hs_k_pk_body(const uint8_t* pk_aff_tl, uint32_t n_pk, uint64_t r) {
  g1_aff p = in_g1(pk_aff_tl);
  g1_jac acc = jac_infinity<fp_t>();
  for (uint32_t k = 0; k < n_pk; ++k) acc = jac_add_aff(acc, p);
  return !jac_is_inf(jac_mul_glv(acc, r));  // Jacobian: the Miller loop takes P projectively
}
void hs_k_miller_body(const uint8_t* p, const uint8_t* q) {
  (void)miller_loop1(jac_from_aff(in_g1(p)), jac_from_aff(in_g2(q)));
}
// the group's signature pair e(-G1, sum r_i sig_i), counted as the one-lane loop
void hs_k_group_miller_body(const uint8_t* q) {
  (void)miller_loop1(jac_from_aff(g1_neg_generator()), jac_from_aff(in_g2(q)));
}
// one complete G2 addition of the group's signature sum
void hs_k_group_add_body(const uint8_t* q, const uint8_t* q2) {
  (void)jac_add(jac_from_aff(in_g2(q)), jac_from_aff(in_g2(q2)));
}
void hs_k_final_body(const uint8_t* f) { (void)fp12_is_one(final_exp(in_fp12(f))); }
// one Fp12 product of the group product in k_final (operands already in Montgomery form)
void hs_k_product_step(const uint8_t* f) {
  const fp12_t a = in_fp12(f);
  hs_count_reset();
  (void)fp12_mul(a, a);
}
#endif

void hs_fp_mul(uint8_t* r, const uint8_t* a, const uint8_t* b) { out_fp(r, fp_mul(in_fp(a), in_fp(b))); }
void hs_fp_add(uint8_t* r, const uint8_t* a, const uint8_t* b) { out_fp(r, fp_add(in_fp(a), in_fp(b))); }
void hs_fp_sub(uint8_t* r, const uint8_t* a, const uint8_t* b) { out_fp(r, fp_sub(in_fp(a), in_fp(b))); }
void hs_fp_neg(uint8_t* r, const uint8_t* a) { out_fp(r, fp_neg(in_fp(a))); }
void hs_fp_inv(uint8_t* r, const uint8_t* a) { out_fp(r, fp_inv(in_fp(a))); }
void hs_fp_half(uint8_t* r, const uint8_t* a) { out_fp(r, fp_half(in_fp(a))); }
int hs_fp_sqrt(uint8_t* r, const uint8_t* a) {
  fp_t s;
  int ok = fp_sqrt(&s, in_fp(a));
  out_fp(r, s);
  return ok;
}
void hs_fp2_mul(uint8_t* r, const uint8_t* a, const uint8_t* b) { out_fp2(r, fp2_mul(in_fp2(a), in_fp2(b))); }
void hs_fp2_sqr(uint8_t* r, const uint8_t* a) { out_fp2(r, fp2_sqr(in_fp2(a))); }
void hs_fp2_inv(uint8_t* r, const uint8_t* a) { out_fp2(r, fp2_inv(in_fp2(a))); }
int hs_fp2_sqrt(uint8_t* r, const uint8_t* a) {
  fp2_t s;
  int ok = fp2_sqrt(&s, in_fp2(a));
  out_fp2(r, s);
  return ok;
}
int hs_fp2_sgn0(const uint8_t* a) { return (int)fp2_sgn0(in_fp2(a)); }
void hs_fp12_mul(uint8_t* r, const uint8_t* a, const uint8_t* b) { out_fp12(r, fp12_mul(in_fp12(a), in_fp12(b))); }
void hs_fp12_sqr(uint8_t* r, const uint8_t* a) { out_fp12(r, fp12_sqr(in_fp12(a))); }
void hs_fp12_inv(uint8_t* r, const uint8_t* a) { out_fp12(r, fp12_inv(in_fp12(a))); }
void hs_fp12_frob(uint8_t* r, const uint8_t* a) { out_fp12(r, fp12_frob(in_fp12(a))); }
void hs_fp12_frob2(uint8_t* r, const uint8_t* a) { out_fp12(r, fp12_frob2(in_fp12(a))); }
void hs_fp12_cyc_sqr(uint8_t* r, const uint8_t* a) { out_fp12(r, fp12_cyclotomic_sqr(in_fp12(a))); }
void hs_fp12_mul_line(uint8_t* r, const uint8_t* f, const uint8_t* l0, const uint8_t* l1, const uint8_t* l3) {
  out_fp12(r, fp12_mul_line(in_fp12(f), in_fp2(l0), in_fp2(l1), in_fp2(l3)));
}
// G2 compressed (96 B) -> test-layout affine (192 B); returns BGV code, 100 = infinity
int hs_g2_decompress(uint8_t* out, const uint8_t* in) {
  g2_aff a;
  bool inf;
  int rc = g2_decompress(&a, &inf, in);
  if (rc) return rc;
  if (inf) return 100;
  out_g2(out, a);
  return 0;
}
void hs_g2_compress(uint8_t* out96, const uint8_t* aff) { g2_compress(out96, in_g2(aff), false); }
int hs_g2_in_subgroup(const uint8_t* aff) { return g2_in_subgroup(jac_from_aff(in_g2(aff))); }
int hs_g2_on_curve(const uint8_t* aff) { return g2_aff_on_curve(in_g2(aff)); }

static int g2_out(uint8_t* out, const g2_jac& j) {
  g2_aff a;
  if (!jac_to_aff(&a, j)) return 0;
  out_g2(out, a);
  return 1;
}
static int g1_out(uint8_t* out, const g1_jac& j) {
  g1_aff a;
  if (!jac_to_aff(&a, j)) return 0;
  out_g1(out, a);
  return 1;
}

int hs_g2_mul_u64(uint8_t* out, const uint8_t* aff, uint64_t k) {
  return g2_out(out, jac_mul_u64(jac_from_aff(in_g2(aff)), k));
}
int hs_g2_add(uint8_t* out, const uint8_t* a, const uint8_t* b) {
  return g2_out(out, jac_add(jac_from_aff(in_g2(a)), jac_from_aff(in_g2(b))));
}
int hs_g2_dbl(uint8_t* out, const uint8_t* a) { return g2_out(out, jac_dbl(jac_from_aff(in_g2(a)))); }
int hs_g2_psi(uint8_t* out, const uint8_t* a) { return g2_out(out, g2_psi(jac_from_aff(in_g2(a)))); }
int hs_g2_clear_cofactor(uint8_t* out, const uint8_t* a) {
  return g2_out(out, g2_clear_cofactor(jac_from_aff(in_g2(a))));
}
int hs_g2_mul_glv(uint8_t* out, const uint8_t* aff, uint64_t k) {
  return g2_out(out, jac_mul_glv(jac_from_aff(in_g2(aff)), k));
}
int hs_g1_mul_glv(uint8_t* out, const uint8_t* aff, uint64_t k) {
  return g1_out(out, jac_mul_glv(jac_from_aff(in_g1(aff)), k));
}
int hs_g1_mul_u64(uint8_t* out, const uint8_t* aff, uint64_t k) {
  return g1_out(out, jac_mul_u64(jac_from_aff(in_g1(aff)), k));
}
int hs_g1_add(uint8_t* out, const uint8_t* a, const uint8_t* b) {
  return g1_out(out, jac_add(jac_from_aff(in_g1(a)), jac_from_aff(in_g1(b))));
}

void hs_hash_to_field(uint8_t* out4x48, const uint8_t* msg, uint32_t len) {
  fp2_t u0, u1;
  hash_to_field_fp2(&u0, &u1, msg, len);
  out_fp2(out4x48, u0);
  out_fp2(out4x48 + 96, u1);
}
void hs_sswu(uint8_t* out, const uint8_t* u) {
  fp2_t x, y;
  sswu_g2(&x, &y, in_fp2(u), fp_sqrt_minus5());
  out_g2(out, g2_aff{x, y});
}
int hs_sswu_iso_jac(uint8_t* out, const uint8_t* u) {
  return g2_out(out, iso_map_g2_jac(sswu_g2_jac(in_fp2(u), fp_sqrt_minus5())));
}
int hs_iso_map(uint8_t* out, const uint8_t* aff) {
  g2_aff a = in_g2(aff);
  return g2_out(out, iso_map_g2(a.x, a.y));
}
int hs_hash_to_g2(uint8_t* out_aff, uint8_t* out_comp96, const uint8_t* msg, uint32_t len) {
  g2_aff a;
  g2_jac h = hash_to_g2(msg, len);
  if (!jac_to_aff(&a, h)) return 0;
  out_g2(out_aff, a);
  g2_compress(out_comp96, a, false);
  return 1;
}

// P (test layout g1) , Q (test layout g2) -> Miller loop value and pairing^3
void hs_miller_loop(uint8_t* out, const uint8_t* p, const uint8_t* q) { out_fp12(out, miller_loop(in_g1(p), in_g2(q))); }
// The bulk path's two-phase Miller loop (k_lines' records, then k_facc's walk) on one pair,
// P and Q Jacobian from affine inputs scaled by z1 / z2 (1: affine)
void hs_miller_two_phase(uint8_t* out, const uint8_t* p, const uint8_t* q, const uint8_t* z1, const uint8_t* z2) {
  const g1_aff pa = in_g1(p);
  const g2_aff qa = in_g2(q);
  const fp_t zp = in_fp(z1);
  const fp2_t zq = in_fp2(z2);
  const fp_t zp2 = fp_sqr(zp);
  const fp2_t zq2 = fp2_sqr(zq);
  const g1_jac P = {fp_mul(pa.x, zp2), fp_mul(pa.y, fp_mul(zp2, zp)), zp};
  const g2_jac Q = {fp2_mul(qa.x, zq2), fp2_mul(qa.y, fp2_mul(zq2, zq)), zq};
  static uint32_t rec[BGV_MILLER_STEPS][BGV_LINE_WORDS];
  miller_lines_walk(&Q, [&](int k, const auto& r) { memcpy(rec[k], &r, sizeof(r)); });
  out_fp12(out, miller_facc_walk(P, [&](int k, auto* r) { memcpy(r, rec[k], sizeof(*r)); }));
}
// the single-pass loop on the same Jacobian inputs
void hs_miller_one_pass(uint8_t* out, const uint8_t* p, const uint8_t* q, const uint8_t* z1, const uint8_t* z2) {
  const g1_aff pa = in_g1(p);
  const g2_aff qa = in_g2(q);
  const fp_t zp = in_fp(z1);
  const fp2_t zq = in_fp2(z2);
  const fp_t zp2 = fp_sqr(zp);
  const fp2_t zq2 = fp2_sqr(zq);
  const g1_jac P = {fp_mul(pa.x, zp2), fp_mul(pa.y, fp_mul(zp2, zp)), zp};
  const g2_jac Q = {fp2_mul(qa.x, zq2), fp2_mul(qa.y, fp2_mul(zq2, zq)), zq};
  out_fp12(out, miller_loop1(P, Q));
}
// The bulk verify path's pairing value for one set: r P by the GLV randomizer (task_pk's
// jac_mul_glv, P left Jacobian), H Jacobian, k_miller's miller_loop1, then final_exp (the
// cube of the pairing) -- pinned against tests/golden/pairing.json
void hs_bulk_pair_value(uint8_t* out, const uint8_t* p, const uint8_t* q, uint64_t word) {
  const g1_jac rp = jac_mul_glv(jac_from_aff(in_g1(p)), word);
  out_fp12(out, final_exp(miller_loop1(rp, jac_from_aff(in_g2(q)))));
}
void hs_final_exp(uint8_t* out, const uint8_t* f) { out_fp12(out, final_exp(in_fp12(f))); }
// team-parallel closing arithmetic (bls_team.h), emulated lane by lane
void hs_team_mul(uint8_t* r, const uint8_t* a, const uint8_t* b) {
  tm_emu_ops o;
  out_fp12(r, tm_emu_to_fp12(o.mul(tm_emu_from_fp12(in_fp12(a)), tm_emu_from_fp12(in_fp12(b)))));
}
void hs_team_sqr(uint8_t* r, const uint8_t* a) {
  tm_emu_ops o;
  out_fp12(r, tm_emu_to_fp12(o.sqr(tm_emu_from_fp12(in_fp12(a)))));
}
void hs_team_frob(uint8_t* r, const uint8_t* a) {
  tm_emu_ops o;
  out_fp12(r, tm_emu_to_fp12(o.frob(tm_emu_from_fp12(in_fp12(a)))));
}
void hs_team_conj(uint8_t* r, const uint8_t* a) {
  tm_emu_ops o;
  out_fp12(r, tm_emu_to_fp12(o.conj(tm_emu_from_fp12(in_fp12(a)))));
}
void hs_team_frob2(uint8_t* r, const uint8_t* a) {
  tm_emu_ops o;
  out_fp12(r, tm_emu_to_fp12(o.frob2(tm_emu_from_fp12(in_fp12(a)))));
}
int hs_team_final_is_one(const uint8_t* f) {
  tm_emu_ops o;
  return tm_final_exp_is_one(o, tm_emu_from_fp12(in_fp12(f)));
}
int hs_final_is_one(const uint8_t* f) { return fp12_is_one(final_exp(in_fp12(f))); }
// the wide (four parts per coefficient) products of the latency path's closing
void hs_team_mul_wide(uint8_t* r, const uint8_t* a, const uint8_t* b) {
  tm_emu_wide_ops o;
  out_fp12(r, tm_emu_to_fp12(o.mul(tm_emu_from_fp12(in_fp12(a)), tm_emu_from_fp12(in_fp12(b)))));
}
void hs_team_sqr_wide(uint8_t* r, const uint8_t* a) {
  tm_emu_wide_ops o;
  out_fp12(r, tm_emu_to_fp12(o.sqr(tm_emu_from_fp12(in_fp12(a)))));
}
int hs_team_final_is_one_wide(const uint8_t* f) {
  tm_emu_wide_ops o;
  return tm_final_exp_is_one(o, tm_emu_from_fp12(in_fp12(f)));
}
// the eight-part products of k_final_fold's final exponentiation
void hs_team_mul_wide8(uint8_t* r, const uint8_t* a, const uint8_t* b) {
  tm_emu_wide8_ops o;
  out_fp12(r, tm_emu_to_fp12(o.mul(tm_emu_from_fp12(in_fp12(a)), tm_emu_from_fp12(in_fp12(b)))));
}
void hs_team_sqr_wide8(uint8_t* r, const uint8_t* a) {
  tm_emu_wide8_ops o;
  out_fp12(r, tm_emu_to_fp12(o.sqr(tm_emu_from_fp12(in_fp12(a)))));
}
int hs_team_final_is_one_wide8(const uint8_t* f) {
  tm_emu_wide8_ops o;
  return tm_final_exp_is_one(o, tm_emu_from_fp12(in_fp12(f)));
}
// the lean eight-part squaring (k_final_fold): value and, part by part, the raw limbs of
// tm_sqr_part8 (returns the number of (c, q) parts that differ)
void hs_team_sqr_wide8_lean(uint8_t* r, const uint8_t* a) {
  tm_emu_wide8_lean_ops o;
  out_fp12(r, tm_emu_to_fp12(o.sqr(tm_emu_from_fp12(in_fp12(a)))));
}
int hs_team_sqr8_lean_diff(const uint8_t* a) {
  const tm_emu_t x = tm_emu_from_fp12(in_fp12(a));
  int bad = 0;
  for (int c = 0; c < BGV_TEAM_COMPS; ++c)
    for (int q = 0; q < 8; ++q) {
      tm_lin_t X, Y;
      tm_sqr_rec8(c, q, &X, &Y);
      const fp_t u = tm_sqr_part8(c, q, x.c), v = tm_sqr_part8_lean(x.c, X, Y);
      for (int l = 0; l < NL; ++l)
        if (u.v[l] != v.v[l]) {
          ++bad;
          break;
        }
    }
  return bad;
}
// the lean four-part squaring (k_miller_wide): parts differing from tm_sqr_part, limb for limb
int hs_team_sqr4_lean_diff(const uint8_t* a) {
  const tm_emu_t x = tm_emu_from_fp12(in_fp12(a));
  int bad = 0;
  for (int c = 0; c < BGV_TEAM_COMPS; ++c)
    for (int q = 0; q < 4; ++q) {
      tm_lin_t X1, Y1, X2, Y2;
      tm_sqr_rec4(c, q, &X1, &Y1, &X2, &Y2);
      const fp_t u = tm_sqr_part(c, q, x.c), v = tm_sqr_part4_lean(x.c, X1, Y1, X2, Y2);
      for (int l = 0; l < NL; ++l)
        if (u.v[l] != v.v[l]) {
          ++bad;
          break;
        }
    }
  return bad;
}
int hs_team_final_is_one_wide8_lean(const uint8_t* f) {
  tm_emu_wide8_lean_ops o;
  return tm_final_exp_is_one(o, tm_emu_from_fp12(in_fp12(f)));
}
// Q handed over in Jacobian form with Z != 1: (l^2 x, l^3 y, l), l = 3 + 5u
static g2_jac jac_scaled(const g2_aff& a) {
  const fp2_t l = {fp_to_mont(fp_t{{3}}), fp_to_mont(fp_t{{5}})};
  const fp2_t l2 = fp2_sqr(l);
  return g2_jac{fp2_mul(a.x, l2), fp2_mul(a.y, fp2_mul(l2, l)), l};
}
// P handed over in Jacobian form with Z != 1 as well: (l^2 x, l^3 y, l), l = 7
static g1_jac g1_scaled(const g1_aff& a) {
  const fp_t l = fp_to_mont(fp_t{{7}});
  const fp_t l2 = fp_sqr(l);
  return g1_jac{fp_mul(a.x, l2), fp_mul(a.y, fp_mul(l2, l)), l};
}
void hs_miller_loop1(uint8_t* out, const uint8_t* p, const uint8_t* q) {
  out_fp12(out, miller_loop1(g1_scaled(in_g1(p)), jac_scaled(in_g2(q))));
}
// the team Miller loop of k_final (bls_team.h tm_miller_loop), emulated lane by lane
void hs_team_miller(uint8_t* out, const uint8_t* p, const uint8_t* q) {
  tm_emu_ops o;
  out_fp12(out, tm_emu_to_fp12(tm_miller_loop<tm_emu_t>(o, g1_scaled(in_g1(p)), jac_scaled(in_g2(q)))));
}
// the latency path's team G2 schedules (bgv_tcurve.h) against the one-lane formulas:
// returns 1 when both the cofactor clearing of a message's two SSWU points and [k] of the
// result agree (as affine points), 0 otherwise; *bad_out = the exceptional-addition flag
int hs_tcurve_check(const uint8_t* msg32, uint64_t k, int* bad_out) {
  fp2_t u0, u1, x, y;
  hash_to_field_fp2(&u0, &u1, msg32, 32);
  sswu_g2(&x, &y, u0, fp_sqrt_minus5());
  const g2_jac q0 = iso_map_g2(x, y);
  sswu_g2(&x, &y, u1, fp_sqrt_minus5());
  const g2_jac q1 = iso_map_g2(x, y);
  // the Jacobian maps (no inversion) give the same points
  if (!jac_eq(q0, iso_map_g2_jac(sswu_g2_jac(u0, fp_sqrt_minus5()))) ||
      !jac_eq(q1, iso_map_g2_jac(sswu_g2_jac(u1, fp_sqrt_minus5()))))
    return 0;
  bool bad;
  const g2_jac h_team = tc_clear_cofactor_host(sswu_g2_jac(u0, fp_sqrt_minus5()), sswu_g2_jac(u1, fp_sqrt_minus5()), &bad);
  const g2_jac h_lane = g2_clear_cofactor(jac_add(q0, q1));
  *bad_out = bad;
  if (!jac_eq(h_team, h_lane)) return 0;
  return jac_eq(tc_mul_glv_host(h_lane, k), jac_mul_glv(h_lane, k)) ? 1 : 0;
}
// the latency path's team loop (bgv_tmiller.h: table-driven twist-point rounds + team Fp12)
// the latency path's G1 schedule (bgv_tg1.h tg1_mul_glv, projective programs) against the
// one-lane jac_mul_glv, P handed in Jacobian with Z != 1: 1 when the points agree
int hs_tg1_check(const uint8_t* p_aff, uint64_t k) {
  const g1_jac p = g1_scaled(in_g1(p_aff));
  return jac_eq(tg1_mul_glv_host(p, k), jac_mul_glv(p, k)) ? 1 : 0;
}
void hs_tmiller(uint8_t* out, const uint8_t* p, const uint8_t* q) {
  out_fp12(out, tm_team_miller_host(g1_scaled(in_g1(p)), jac_scaled(in_g2(q))));
}
// k_miller_wide: four-part round instructions and the wide Fp12 products
void hs_tmiller_wide(uint8_t* out, const uint8_t* p, const uint8_t* q) {
  tmp_host_wide() = true;
  out_fp12(out, tm_team_miller_host<tm_emu_wide_ops>(g1_scaled(in_g1(p)), jac_scaled(in_g2(q))));
  tmp_host_wide() = false;
}
// the point programs' rounds as four-part instructions (k_prep_wide) from now on, or not
void hs_set_wide_rounds(int on) { tmp_host_wide() = on != 0; }
void hs_team_mul_line(uint8_t* r, const uint8_t* f, const uint8_t* l0, const uint8_t* l1, const uint8_t* l3) {
  tm_emu_ops o;
  out_fp12(r, tm_emu_to_fp12(o.mul_line(tm_emu_from_fp12(in_fp12(f)), in_fp2(l0), in_fp2(l1), in_fp2(l3))));
}
void hs_team_mul_line_wide(uint8_t* r, const uint8_t* f, const uint8_t* l0, const uint8_t* l1, const uint8_t* l3) {
  tm_emu_wide_ops o;
  out_fp12(r, tm_emu_to_fp12(o.mul_line(tm_emu_from_fp12(in_fp12(f)), in_fp2(l0), in_fp2(l1), in_fp2(l3))));
}
void hs_team_mul_line_wide8(uint8_t* r, const uint8_t* f, const uint8_t* l0, const uint8_t* l1, const uint8_t* l3) {
  tm_emu_wide8_ops o;
  out_fp12(r, tm_emu_to_fp12(o.mul_line(tm_emu_from_fp12(in_fp12(f)), in_fp2(l0), in_fp2(l1), in_fp2(l3))));
}
// one set through the device equation: k_prep (r pk affine, r sig Jacobian), k_miller
// (e(r pk, H)), the group's team loop e(-G1, r sig), the product and the team final check
int hs_verify_one(const uint8_t* pk_aff, const uint8_t* h_aff, const uint8_t* sig_aff, uint64_t r) {
  const g1_jac pa = jac_mul_glv(jac_from_aff(in_g1(pk_aff)), r);
  if (jac_is_inf(pa)) return 0;
  const g2_jac rs = jac_mul_glv(jac_from_aff(in_g2(sig_aff)), r);
  tm_emu_ops o;
  const tm_emu_t f = tm_emu_from_fp12(miller_loop1(pa, jac_from_aff(in_g2(h_aff))));
  const tm_emu_t g = tm_miller_loop<tm_emu_t>(o, jac_from_aff(g1_neg_generator()), rs);
  return tm_final_exp_is_one(o, o.mul(f, g));
}

int hs_g1_decompress(uint8_t* out, const uint8_t* in48) {
  g1_aff a;
  bool inf;
  int rc = g1_decompress(&a, &inf, in48);
  if (rc) return rc;
  if (inf) return 100;
  out_g1(out, a);
  return 0;
}
void hs_g1_serialize(uint8_t* out96, const uint8_t* aff) { g1_serialize(out96, in_g1(aff), false); }
// ---- deferred-reduction Fp2 products (bls_wide.h) against the fully reduced Karatsuba ----
// n random operand pairs per bound pair and the extreme ones (every limb at its bound, the top
// limb as high as the value bound allows, zero); both results reduced and compared mod p.
extern "C++" {
static uint64_t hs_rng_state;
static uint64_t hs_rng() {
  hs_rng_state ^= hs_rng_state << 13;
  hs_rng_state ^= hs_rng_state >> 7;
  hs_rng_state ^= hs_rng_state << 17;
  return hs_rng_state;
}
template <uint64_t L, uint64_t V>
static lz<L, V> hs_lz(int kind) {
  lz<L, V> r;
  const uint32_t top = (uint32_t)((V - 1) * (lzc::P13 + 1) < L ? (V - 1) * (lzc::P13 + 1) : L);
  for (int i = 0; i < NL; ++i) {
    if (kind == 0) r.v[i] = (uint32_t)(hs_rng() % (L + 1));
    else if (kind == 1) r.v[i] = (uint32_t)L;
    else r.v[i] = 0;
  }
  r.v[NL - 1] = kind == 0 ? (uint32_t)(hs_rng() % (top + 1)) : (kind == 1 ? top : 0);
  LZ_CHECK(r, "hs_lz");
  return r;
}
template <uint64_t L, uint64_t V>
static bool hs_same(const lz<L, V>& a, const lz<LMASK, 2>& b) {
  const fp_t x = fp_canon(lz_out(lz_norm(a))), y = fp_canon(lz_out(b));
  return memcmp(x.v, y.v, sizeof(x.v)) == 0;
}
template <uint64_t LA, uint64_t VA, uint64_t LB, uint64_t VB>
static int hs_wide_pair(int n) {
  int bad = 0;
  for (int t = 0; t < n + 9; ++t) {
    const int ka = t < n ? 0 : (t - n) / 3, kb = t < n ? 0 : (t - n) % 3;
    const lz2<LA, VA> a{hs_lz<LA, VA>(ka), hs_lz<LA, VA>(kb)};
    const lz2<LB, VB> b{hs_lz<LB, VB>(kb), hs_lz<LB, VB>(ka)};
    const auto w = lz2_mul_w(a, b);
    const auto c = lz2_red(lz2_mul_c(a, b));
    bad += !hs_same(w.c0, c.c0) || !hs_same(w.c1, c.c1);
    const auto m = lz2_mul_fp_w(a, b.c0);
    const auto mc = lz2_mul_fp_c(a, b.c0);
    bad += !hs_same(m.c0, mc.c0) || !hs_same(m.c1, mc.c1);
  }
  return bad;
}
}  // extern "C++"
int hs_wide_check(int n, uint64_t seed) {
  hs_rng_state = seed | 1;
  int bad = 0;
  bad += hs_wide_pair<LMASK, 2, LMASK, 2>(n);
  bad += hs_wide_pair<LMASK, 3, LMASK, 3>(n);
  bad += hs_wide_pair<(1u << 29) - 1, 4, (1u << 29) - 1, 4>(n);
  bad += hs_wide_pair<(1u << 29) - 1, 40, LMASK, 8>(n);
  bad += hs_wide_pair<LMASK, 8, (1u << 29) - 1, 8>(n);
  for (int t = 0; t < n + 3; ++t) {  // the squaring at its limb bound
    const int k = t < n ? 0 : t - n;
    const lz2<BGV_WSQR_LIMB, BGV_WSQR_V> a{hs_lz<BGV_WSQR_LIMB, BGV_WSQR_V>(k), hs_lz<BGV_WSQR_LIMB, BGV_WSQR_V>(k == 0 ? 0 : 2 - k / 2)};
    const auto w = lz2_sqr_w(a);
    const auto c = lz2_sqr_c(a);
    bad += !hs_same(w.c0, c.c0) || !hs_same(w.c1, c.c1);
  }
  return bad;
}
}
