// Pairing kernels of a verify call (gfx950): the groups' signature sums and the Miller
// loops of the randomized batch equation of blst's verifyMultipleAggregateSignatures
// (packages/beacon-node/src/chain/bls/maybeBatch.ts:18-25):
//   prod_i e(r_i pk_i, H(m_i)) * e(-G1, sum_i r_i sig_i) == 1
//
//   k_gsum     per device group (a team of 16 lanes): S_g = sum of the group's r_i sig_i
//   k_miller   f_i = MillerLoop(r_i pk_i, H(m_i)), one pair per lane, and on extra lanes
//              one per group g_g = MillerLoop(-G1, S_g)
//   k_gpair    retry rounds: the parts' signature pairs alone
//   k_miller_team  the latency path for small calls: the same pairs, one per team of 16
//              lanes (bgv_tmiller.h), ~10x lower latency per pair than one lane
#include "bgv_device.h"
#include "bgv_team_dev.h"
#include "bgv_tmiller.h"
#include "bgv_tround_dev.h"

static __constant__ uint8_t kTmProg[TMP_TABLE_BYTES] = TMP_TABLE_INIT;


extern "C" {

// Lanes [0, nslots): f_i = MillerLoop(r pk, H(m)), 1 for slots that do not take part.
// Lanes [nslots, nslots + ngroups): the group's signature pair MillerLoop(-G1, S_g) (1 for
// an infinite S_g), so the group pairs run beside the set pairs instead of after them.
// -G1 in Jacobian form, in memory for miller_loop1m
static __device__ const g1_jac kNegG1Jac = {{BGV_G1X}, {BGV_NEG_G1Y}, {BGV_ONE}};

__device__ __forceinline__ fp12_t group_pair(const g2_jac* S) {
  return jac_is_inf(*S) ? fp12_one() : miller_loop1m(&kNegG1Jac, S);
}

__global__ void BGV_KATTR k_miller(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                   const g1_jac* __restrict__ rpk, const g2_jac* __restrict__ h,
                                   const int32_t* __restrict__ sig_status, const int32_t* __restrict__ pk_status,
                                   fp12_t* __restrict__ f, uint32_t ngroups, const g2_jac* __restrict__ gsum,
                                   fp12_t* __restrict__ gpair) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < nslots) {
    fp12_t r = fp12_one();
    if (slot_live(slots[s], sig_status[s], pk_status[s])) r = miller_loop1m(rpk + s, h + slots[s].hsrc);
    f[s] = r;
  } else if (s - nslots < ngroups) {
    gpair[s - nslots] = group_pair(gsum + (s - nslots));
  }
}

// retry rounds: the signature pairs of the round's parts alone
__global__ void BGV_KATTR k_gpair(uint32_t ngroups, const g2_jac* __restrict__ gsum, fp12_t* __restrict__ gpair) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ngroups) gpair[g] = group_pair(gsum + g);
}

}  // extern "C"
// A lane's share of sum_k (k + 1) P_k over slots k = c + 16 t (t = 0..3) of its team:
// (c + 1) A + 16 B with A = sum_t P_t and B = sum_t t P_t = S1 + S2 + S3, the suffix sums
// S_t = sum_{t' >= t} P_t' taken from t = 3 down (no array of points: the kernel's stack frame
// stays that of its point additions).  load(t) returns P_t (infinity for a dead or absent slot).
template <class P, class Load>
__device__ P weighted_lane_sum(int c, Load load) {
  using F = decltype(P{}.x);
  P S = jac_infinity<F>(), B = jac_infinity<F>();
  BGV_NO_UNROLL for (int t = 3; t >= 0; --t) {
    S = jac_add(S, load(t));
    if (t >= 1) B = jac_add(B, S);
  }
  BGV_UNROLL for (int i = 0; i < 4; ++i) B = jac_dbl(B);  // 16 B
  P r = jac_infinity<F>();
  const uint32_t w = (uint32_t)c + 1;  // <= 16: five bits, the same loop shape on every lane
  BGV_NO_UNROLL for (int bit = 4; bit >= 0; --bit) {
    r = jac_dbl(r);
    const P ra = jac_add(r, S);
    r = ((w >> bit) & 1) ? ra : r;
  }
  return jac_add(r, B);
}
extern "C" {

// S_g = sum of r_i sig_i over a group's live, non-infinity signatures (blst skips an
// infinity signature in the accumulator).  A team of 16 lanes per group: lane c sums
// every 16th slot, then a 4-level ds_swizzle butterfly; the team leader writes S_g.
// A uniform group (BGV_GROUP_UNIFORM: a first-pass group, or a retry test inside one) also sums
// its live slots' r_i pk_i into gpk: its set pairs are then one pair e(gpk, H) (the same slots
// k_facc would pair).
__global__ void __launch_bounds__(64) k_gsum(const bgv_dgroup* __restrict__ groups, uint32_t ngroups,
                                             const bgv_dslot* __restrict__ slots, const g2_jac* __restrict__ rsig,
                                             const int32_t* __restrict__ sig_status,
                                             const int32_t* __restrict__ pk_status, g2_jac* __restrict__ gsum,
                                             const g1_jac* __restrict__ rpk, g1_jac* __restrict__ gpk) {
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const uint32_t gi = blockIdx.x * BGV_FINAL_TEAMS + team;
  const bgv_dgroup g = groups[gi < ngroups ? gi : ngroups - 1];
  if (g.flags & BGV_GROUP_WEIGHTED) return;  // k_gsum_w's (uniform over the team)
  g2_jac acc = jac_infinity<fp2_t>();
  for (uint32_t k = (uint32_t)c; k < g.n_slots; k += BGV_TEAM) {
    if (!grp_has(g, k)) continue;
    const uint32_t s = g.first_slot + k;
    const int32_t ss = sig_status[s];
    if (ss == BGV_ST_OK && slot_live(slots[s], ss, pk_status[s])) acc = jac_add(acc, rsig[s]);
  }
  if (gpk && (g.flags & BGV_GROUP_UNIFORM)) {  // uniform over the team
    g1_jac pa = jac_infinity<fp_t>();
    for (uint32_t k = (uint32_t)c; k < g.n_slots; k += BGV_TEAM) {
      if (!grp_has(g, k)) continue;
      const uint32_t s = g.first_slot + k;
      if (slot_live(slots[s], sig_status[s], pk_status[s])) pa = jac_add(pa, rpk[s]);
    }
    pa = jac_add(pa, point_xor<8>(pa));
    pa = jac_add(pa, point_xor<4>(pa));
    pa = jac_add(pa, point_xor<2>(pa));
    pa = jac_add(pa, point_xor<1>(pa));
    if (gi < ngroups && c == 0) gpk[gi] = pa;
  }
  acc = jac_add(acc, point_xor<8>(acc));
  acc = jac_add(acc, point_xor<4>(acc));
  acc = jac_add(acc, point_xor<2>(acc));
  acc = jac_add(acc, point_xor<1>(acc));
  if (gi < ngroups && c == 0) gsum[gi] = acc;
}

// The weighted tests' sums (BGV_GROUP_WEIGHTED: a whole uniform group, slot k weighted by k + 1):
// sum (k + 1) r_k sig_k into gsum and sum (k + 1) r_k pk_k into gpk, one team of 16 lanes per
// group as k_gsum.  A kernel of its own: its doublings would give k_gsum a 3 KB stack frame
// (256 B alone).
__global__ void __launch_bounds__(64) k_gsum_w(const bgv_dgroup* __restrict__ groups, uint32_t ngroups,
                                               const bgv_dslot* __restrict__ slots, const g2_jac* __restrict__ rsig,
                                               const int32_t* __restrict__ sig_status,
                                               const int32_t* __restrict__ pk_status, g2_jac* __restrict__ gsum,
                                               const g1_jac* __restrict__ rpk, g1_jac* __restrict__ gpk) {
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const uint32_t gi = blockIdx.x * BGV_FINAL_TEAMS + team;
  const bgv_dgroup g = groups[gi < ngroups ? gi : ngroups - 1];
  if (!(g.flags & BGV_GROUP_WEIGHTED)) return;  // k_gsum's (uniform over the team)
  auto live_at = [&](int t, bool* sig_ok) {  // slot t of the lane takes part; *sig_ok: its signature too
    const uint32_t k = (uint32_t)c + BGV_TEAM * t;
    *sig_ok = false;
    if (k >= g.n_slots || !grp_has(g, k)) return false;
    const uint32_t s = g.first_slot + k;
    const int32_t ss = sig_status[s];
    const bool live = slot_live(slots[s], ss, pk_status[s]);
    *sig_ok = live && ss == BGV_ST_OK;
    return live;
  };
  g2_jac acc = weighted_lane_sum<g2_jac>(c, [&](int t) {
    bool ok;
    live_at(t, &ok);
    return ok ? rsig[g.first_slot + c + BGV_TEAM * t] : jac_infinity<fp2_t>();
  });
  acc = jac_add(acc, point_xor<8>(acc));
  acc = jac_add(acc, point_xor<4>(acc));
  acc = jac_add(acc, point_xor<2>(acc));
  acc = jac_add(acc, point_xor<1>(acc));
  if (gi < ngroups && c == 0) gsum[gi] = acc;
  if (g.flags & BGV_GROUP_UNIFORM) {  // the pubkey side of a test with one root (team-uniform)
    g1_jac pa = weighted_lane_sum<g1_jac>(c, [&](int t) {
      bool ok;
      return live_at(t, &ok) ? rpk[g.first_slot + c + BGV_TEAM * t] : jac_infinity<fp_t>();
    });
    pa = jac_add(pa, point_xor<8>(pa));
    pa = jac_add(pa, point_xor<4>(pa));
    pa = jac_add(pa, point_xor<2>(pa));
    pa = jac_add(pa, point_xor<1>(pa));
    if (gi < ngroups && c == 0 && gpk) gpk[gi] = pa;
  }
}

// One Miller loop per team of 16 lanes: pairs [0, nslots) are the sets' e(r pk, H(m)),
// pairs [nslots, nslots + ngroups) the groups' e(-G1, S_g).  The twist point runs the
// generated rounds (bgv_tmiller_prog.h) on the team's LDS slots, the Fp12 accumulator is
// coefficient-parallel.  Teams past the end (and pairs that take no part) compute on
// zeros and store 1 or nothing, so every lane reaches every barrier.
// Pairs [nslots + ngroups, + npk) (retry rounds with uniform groups): pair j is test t =
// upk[j]'s pubkey-sum pair e(gpk_t, H of its root) into gpkp_t (groups[t] is BGV_GROUP_UNIFORM).
#define BGV_MTEAM_ARGS                                                                                      \
  const bgv_dslot *__restrict__ slots, uint32_t nslots, const g1_jac *__restrict__ rpk,                      \
      const g2_jac *__restrict__ h, const int32_t *__restrict__ sig_status, const int32_t *__restrict__ pk_status, \
      fp12_t *__restrict__ f, uint32_t ngroups, const g2_jac *__restrict__ gsum, fp12_t *__restrict__ gpair,   \
      const bgv_dgroup *__restrict__ groups, const uint32_t *__restrict__ upk, uint32_t npk,                   \
      const g1_jac *__restrict__ gpk, fp12_t *__restrict__ gpkp
}  // extern "C"
__device__ __forceinline__ void miller_team_body(BGV_MTEAM_ARGS) {
  __shared__ uint8_t prog[TMP_TABLE_BYTES];
  __shared__ fp_t S[BGV_FINAL_TEAMS][TMP_NSLOT];
  __shared__ fp_t lds[BGV_FINAL_TEAMS][2 * BGV_TEAM_COMPS];
  for (int i = threadIdx.x; i < TMP_TABLE_BYTES; i += 64) prog[i] = kTmProg[i];
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const int cc = c < BGV_TEAM_COMPS ? c : c - 4;
  const uint32_t total = nslots + ngroups + npk;
  const uint32_t u = blockIdx.x * BGV_FINAL_TEAMS + team;
  const uint32_t uu = u < total ? u : total - 1;
  const bool set_pair = uu < nslots, pk_pair = uu >= nslots + ngroups;
  const g1_jac* pk_p = nullptr;  // P of a set pair or a pubkey-sum pair
  bool live;
  const fp_t* qsrc;
  fp12_t* dst;
  if (set_pair) {
    live = slot_live(slots[uu], sig_status[uu], pk_status[uu]);
    qsrc = reinterpret_cast<const fp_t*>(h + slots[uu].hsrc);  // H of the slot's signing root
    pk_p = rpk + uu;
    dst = f + uu;
  } else if (!pk_pair) {
    qsrc = reinterpret_cast<const fp_t*>(gsum + (uu - nslots));
    live = !jac_is_inf(gsum[uu - nslots]);
    dst = gpair + (uu - nslots);
  } else {
    const uint32_t t = upk[uu - nslots - ngroups];
    const bgv_dgroup G = groups[t];
    qsrc = reinterpret_cast<const fp_t*>(h + slots[G.first_slot].hsrc);  // the group's one root
    live = !jac_is_inf(gpk[t]);
    pk_p = gpk + t;
    dst = gpkp + t;
  }
  fp_t* Sm = S[team];
  if (c < 6) {
    const fp_t v = live ? qsrc[c] : fp_zero();
    Sm[TMP_S_QX + c] = v;
    Sm[TMP_S_BANK0 + c] = v;
  } else if (c < 9) {
    // P in Jacobian form (bls_pairing.h miller_p): -X Z, Y, Z^3
    const g1_jac P = pk_p ? *pk_p : jac_from_aff(g1_neg_generator());
    const fp_t v = c == 6 ? fp_neg(fp_mul(P.x, P.z)) : (c == 7 ? P.y : fp_mul(fp_sqr(P.z), P.z));
    Sm[c == 6 ? TMP_S_XN : (c == 7 ? TMP_S_YP : TMP_S_ZP3)] = live ? v : fp_zero();
  } else if (c == 9) {
    Sm[TMP_S_ONE] = fp_one();
  }
  __syncthreads();
  auto run = [&](int off) {
    int pos = off;
    const int nr = prog[pos++];
    for (int r = 0; r < nr; ++r) {
      const int T = prog[pos], M = prog[pos + 1];
      pos += 2;
      const int rb = tmp_rec_bytes(T, M);
      int out;
      const fp_t v = tmp_lane_any(Sm, prog + pos + c * rb, T, M, &out);
      Sm[out] = v;  // no slot is read and written in one round (tools/gen_tmiller.py)
      __syncthreads();
      pos += BGV_TEAM * rb;
    }
  };
  tm_dev_ops o{lds[team], lds[team] + BGV_TEAM_COMPS, c, cc};
  run(TMP_INIT);
  run(TMP_DBL0);
  int bank = 1;
  fp2_t l0 = {Sm[TMP_S_L0], Sm[TMP_S_L0 + 1]}, l1 = {Sm[TMP_S_L1], Sm[TMP_S_L1 + 1]},
        l3 = {Sm[TMP_S_L3], Sm[TMP_S_L3 + 1]};
  fp_t x = o.line(l0, l1, l3);
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if (tmp_add_at(i)) {
      run(bank ? TMP_ADD1 : TMP_ADD0);
      bank ^= 1;
      l0 = fp2_t{Sm[TMP_S_L0], Sm[TMP_S_L0 + 1]};
      l1 = fp2_t{Sm[TMP_S_L1], Sm[TMP_S_L1 + 1]};
      l3 = fp2_t{Sm[TMP_S_L3], Sm[TMP_S_L3 + 1]};
      x = o.mul_line(x, l0, l1, l3);
    }
    x = o.sqr(x);
    run(bank ? TMP_DBL1 : TMP_DBL0);
    bank ^= 1;
    l0 = fp2_t{Sm[TMP_S_L0], Sm[TMP_S_L0 + 1]};
    l1 = fp2_t{Sm[TMP_S_L1], Sm[TMP_S_L1 + 1]};
    l3 = fp2_t{Sm[TMP_S_L3], Sm[TMP_S_L3 + 1]};
    x = o.mul_line(x, l0, l1, l3);
  }
  x = o.conj(x);
  if (u < total && c < BGV_TEAM_COMPS && dst)
    reinterpret_cast<fp_t*>(dst)[tm_fp_index(cc)] = live ? x : (cc == 0 ? fp_one() : fp_zero());
}
extern "C" {
__global__ void __launch_bounds__(64) k_miller_team(BGV_MTEAM_ARGS) {
  miller_team_body(slots, nslots, rpk, h, sig_status, pk_status, f, ngroups, gsum, gpair, groups, upk, npk, gpk,
                   gpkp);
}

// The same pairs with one pair per block for the smallest calls, on two waves that run the
// loop's two chains side by side: wave 0 the twist-point rounds of k_miller_team as
// four-part instructions (bgv_tround_dev.h), wave 1 the Fp12 accumulator with the wide
// products (bgv_team_dev.h tm_wide_ops: each coefficient's double-width products split over
// four lanes).  The point rounds of step i need nothing from the accumulator, so wave 0
// computes step i's lines while wave 1 applies step i + 1's (square, line products); the
// lines pass through a two-entry LDS ring with one block barrier per step, and a step costs
// the longer of the two chains instead of their sum.  Same formulas, same field element as
// k_miller_team.  rsig non-null (bgv_sig_pairs): blocks [nslots, 2 nslots) pair the slots'
// own r_i sig_i with -G1 into fsig instead of pairing group sums.
__global__ void __launch_bounds__(128) k_miller_wide(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                                     const g1_jac* __restrict__ rpk, const g2_jac* __restrict__ h,
                                                     const int32_t* __restrict__ sig_status,
                                                     const int32_t* __restrict__ pk_status, fp12_t* __restrict__ f,
                                                     uint32_t ngroups, const g2_jac* __restrict__ gsum,
                                                     fp12_t* __restrict__ gpair, const g2_jac* __restrict__ rsig,
                                                     fp12_t* __restrict__ fsig) {
  __shared__ uint8_t prog[TMP_TABLE_BYTES];
  __shared__ fp_t Sm[TMP_NSLOT];
  __shared__ fp_t WA[BGV_TEAM_COMPS], WB[BGV_TEAM_COMPS], WP[4 * BGV_TEAM_COMPS], RP[64];
  __shared__ fp_t LR[2][2][6];  // [step & 1][addition line, doubling line][l0, l1, l3 as Fp pairs]
  for (int i = threadIdx.x; i < TMP_TABLE_BYTES; i += 128) prog[i] = kTmProg[i];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t uu = blockIdx.x;  // grid = exactly nslots + ngroups blocks
  const bool set_pair = uu < nslots;
  bool live;
  const fp_t* qsrc;
  const uint32_t j = uu - nslots;
  if (set_pair) {
    live = slot_live(slots[uu], sig_status[uu], pk_status[uu]);
    qsrc = reinterpret_cast<const fp_t*>(h + slots[uu].hsrc);
  } else if (rsig) {  // the slot's own signature pair (an infinity signature is skipped: 1)
    live = slot_live(slots[j], sig_status[j], pk_status[j]) && sig_status[j] == BGV_ST_OK;
    qsrc = reinterpret_cast<const fp_t*>(rsig + j);
  } else {
    qsrc = reinterpret_cast<const fp_t*>(gsum + j);
    live = !jac_is_inf(gsum[j]);
  }
  if (w == 0) {
    if (lane < 6) {
      const fp_t v = live ? qsrc[lane] : fp_zero();
      Sm[TMP_S_QX + lane] = v;
      Sm[TMP_S_BANK0 + lane] = v;
    } else if (lane < 9) {
      const g1_jac P = set_pair ? rpk[uu] : jac_from_aff(g1_neg_generator());
      const fp_t v = lane == 6 ? fp_neg(fp_mul(P.x, P.z)) : (lane == 7 ? P.y : fp_mul(fp_sqr(P.z), P.z));
      Sm[lane == 6 ? TMP_S_XN : (lane == 7 ? TMP_S_YP : TMP_S_ZP3)] = live ? v : fp_zero();
    } else if (lane == 9) {
      Sm[TMP_S_ONE] = fp_one();
    }
  }
  __syncthreads();
  tr_wide_engine eng{prog, Sm, RP, tr_wide_lane_c(lane), tr_wide_lane_q(lane), false};
  // wave 0: the line of the last program run into ring entry (r, k)
  auto post = [&](int r, int k) {
    if (lane < 6) LR[r][k][lane] = Sm[(lane < 2 ? TMP_S_L0 : (lane < 4 ? TMP_S_L1 - 2 : TMP_S_L3 - 4)) + lane];
  };
  // the Fp12 accumulator's squarings from the lane's operand recipes (bls_team.h tm_sqr_rec4)
  tm_wide4_lean_ops o;
  o.A = WA;
  o.B = WB;
  o.P = WP;
  o.c = lane % BGV_TEAM_COMPS;
  o.q = lane / BGV_TEAM_COMPS;
  tm_sqr_rec4(o.c, o.q < 4 ? o.q : 3, &o.x1, &o.y1, &o.x2, &o.y2);
  auto ln = [&](int r, int k, fp2_t* l0, fp2_t* l1, fp2_t* l3) {
    const fp_t* L = LR[r][k];
    *l0 = fp2_t{L[0], L[1]};
    *l1 = fp2_t{L[2], L[3]};
    *l3 = fp2_t{L[4], L[5]};
  };
  fp_t x;
  if (w == 0) {
    eng.run(TMP_INIT);
    eng.run(TMP_DBL0);
    post(0, 1);
  }
  __syncthreads();
  if (w == 1) {
    fp2_t l0, l1, l3;
    ln(0, 1, &l0, &l1, &l3);
    x = o.line(l0, l1, l3);
  }
  // step i (61..0): wave 0 computes its lines into ring entry i & 1 while wave 1 applies step
  // i + 1's from entry (i + 1) & 1; the barrier ends both
  int bank = 1;
  BGV_NO_UNROLL for (int i = 61; i >= -1; --i) {
    if (w == 0) {
      if (i >= 0) {
        if (tmp_add_at(i)) {
          eng.run(bank ? TMP_ADD1 : TMP_ADD0);
          bank ^= 1;
          post(i & 1, 0);
        }
        eng.run(bank ? TMP_DBL1 : TMP_DBL0);
        bank ^= 1;
        post(i & 1, 1);
      }
    } else if (i < 61) {
      const int s = i + 1, r = s & 1;
      fp2_t l0, l1, l3;
      if (tmp_add_at(s)) {
        ln(r, 0, &l0, &l1, &l3);
        x = o.mul_line(x, l0, l1, l3);
      }
      x = o.sqr(x);
      ln(r, 1, &l0, &l1, &l3);
      x = o.mul_line(x, l0, l1, l3);
    }
    __syncthreads();
  }
  if (w == 1) {
    x = o.conj(x);
    if (lane < BGV_TEAM_COMPS) {
      fp12_t* dst = set_pair ? f + uu : (rsig ? fsig + j : gpair + j);
      reinterpret_cast<fp_t*>(dst)[tm_fp_index(lane)] = live ? x : (lane == 0 ? fp_one() : fp_zero());
    }
  }
}

}  // extern "C"

bool bgv_sig_pairs(const bgv_dev_batch& b) {
  return bgv_use_latency(b, b.nslots + b.ngroups) && b.nslots <= BGV_PREP_WIDE_MAX;
}

static void launch_miller_latency(const bgv_dev_batch& b, uint32_t nslots, uint32_t ngroups, hipStream_t st) {
  const uint32_t total = nslots + ngroups;
  if (total <= BGV_MILLER_WIDE_MAX)
    hipLaunchKernelGGL(k_miller_wide, dim3(total), dim3(128), 0, st, b.slots, nslots, b.rpk, b.h, b.sig_status,
                       b.pk_status, b.f, ngroups, b.gsum, b.gpair, static_cast<const g2_jac*>(nullptr),
                       static_cast<fp12_t*>(nullptr));
  else
    hipLaunchKernelGGL(k_miller_team, dim3(nblk(total, BGV_FINAL_TEAMS)), dim3(64), 0, st, b.slots, nslots, b.rpk,
                       b.h, b.sig_status, b.pk_status, b.f, ngroups, b.gsum, b.gpair,
                       static_cast<const bgv_dgroup*>(nullptr), static_cast<const uint32_t*>(nullptr), 0u,
                       static_cast<const g1_jac*>(nullptr), static_cast<fp12_t*>(nullptr));
}

// lanes of one k_miller round: one wave of 64 on each SIMD (MI355X: 256 CUs x 4 SIMDs)
static uint32_t miller_round_lanes() {
  static const uint32_t lanes = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return (uint32_t)cus * 4u * 64u;
  }();
  return lanes;
}

// BGV_MILLER_1PASS=1: the single-pass k_miller (one lane holds f, T and P) instead of
// k_lines + k_facc, for A/B measurements; it needs no line records
bool bgv_single_pass_miller() {
  static const bool v = [] {
    const char* e = getenv("BGV_MILLER_1PASS");
    return e && atoi(e) > 0;
  }();
  return v;
}

hipError_t bgv_launch_miller(const bgv_dev_batch& b, const bgv_streams& s) {
  const uint32_t n = b.nslots;
  if (n == 0) return hipSuccess;
  if (bgv_sig_pairs(b)) {  // no group sums: every slot's own signature pair beside its set pair
    hipLaunchKernelGGL(k_miller_wide, dim3(2 * n), dim3(128), 0, s.main, b.slots, n, b.rpk, b.h, b.sig_status,
                       b.pk_status, b.f, n, b.gsum, b.gpair, b.rsig, b.fsig);
    BGV_MARK(3);
    return hipGetLastError();
  }
  // the groups' signature sums, then set pairs and group pairs in one launch
  hipLaunchKernelGGL(k_gsum, dim3(nblk(b.ngroups, BGV_FINAL_TEAMS)), dim3(64), 0, s.main, b.groups, b.ngroups,
                     b.slots, b.rsig, b.sig_status, b.pk_status, b.gsum, static_cast<const g1_jac*>(b.rpk), b.gpk);
  BGV_MARK(2);
  const uint32_t R = miller_round_lanes();
  if (bgv_use_latency(b, n + b.ngroups)) {
    launch_miller_latency(b, n, b.ngroups, s.main);
  } else if (b.path != BGV_PATH_BULK && b.ngroups <= bgv_latency_max() &&
             (n + b.ngroups + R - 1) / R > (n + R - 1) / R && !b.uniform) {
    // the group pairs on extra k_facc lanes would open one more round of one wave per SIMD
    // (131,072 sets + 2,048 groups: 3 rounds instead of 2); run them on teams instead.  Not
    // with uniform groups: their slot lanes exit at once, so no round is full anyway
    hipLaunchKernelGGL(k_miller_team, dim3(nblk(b.ngroups, BGV_FINAL_TEAMS)), dim3(64), 0, s.main, b.slots, 0u,
                       b.rpk, b.h, b.sig_status, b.pk_status, b.f, b.ngroups, b.gsum, b.gpair,
                       static_cast<const bgv_dgroup*>(nullptr), static_cast<const uint32_t*>(nullptr), 0u,
                       static_cast<const g1_jac*>(nullptr), static_cast<fp12_t*>(nullptr));
    if (bgv_single_pass_miller())
      hipLaunchKernelGGL(k_miller, dim3(nblk(n, 64)), dim3(64), 0, s.main, b.slots, n, b.rpk, b.h, b.sig_status,
                         b.pk_status, b.f, 0u, b.gsum, b.gpair);
    else if (hipError_t e = bgv_launch_miller_bulk(b, 0u, s.main); e != hipSuccess)
      return e;
  } else if (bgv_single_pass_miller()) {
    hipLaunchKernelGGL(k_miller, dim3(nblk(n + b.ngroups, 64)), dim3(64), 0, s.main, b.slots, n, b.rpk, b.h,
                       b.sig_status, b.pk_status, b.f, b.ngroups, b.gsum, b.gpair);
  } else if (hipError_t e = bgv_launch_miller_bulk(b, b.ngroups, s.main); e != hipSuccess) {
    return e;
  }
  BGV_MARK(3);
  return hipGetLastError();
}

hipError_t bgv_launch_sets(const bgv_dev_batch& b, const bgv_streams& s) {
  hipError_t e = bgv_launch_prep(b, s);
  return e != hipSuccess ? e : bgv_launch_miller(b, s);
}

// retry rounds over parts of failed groups: the parts' signature sums and pairs; with uniform
// groups (b.uniform) also the pubkey sums and pubkey-sum pairs of the tests flagged
// BGV_GROUP_UNIFORM (their slots have no own pair: bgv_api.cpp call_build_parts)
hipError_t bgv_launch_gpairs(const bgv_dev_batch& b, hipStream_t st) {
  if (b.ngroups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gsum, dim3(nblk(b.ngroups, BGV_FINAL_TEAMS)), dim3(64), 0, st, b.groups, b.ngroups, b.slots,
                     b.rsig, b.sig_status, b.pk_status, b.gsum, static_cast<const g1_jac*>(b.rpk),
                     b.uniform ? static_cast<g1_jac*>(b.gpk) : static_cast<g1_jac*>(nullptr));
  if (b.weighted)
    hipLaunchKernelGGL(k_gsum_w, dim3(nblk(b.ngroups, BGV_FINAL_TEAMS)), dim3(64), 0, st, b.groups, b.ngroups,
                       b.slots, b.rsig, b.sig_status, b.pk_status, b.gsum, static_cast<const g1_jac*>(b.rpk),
                       static_cast<g1_jac*>(b.gpk));
  if (b.uniform)
    hipLaunchKernelGGL(k_miller_team, dim3(nblk(b.ngroups + b.npk, BGV_FINAL_TEAMS)), dim3(64), 0, st, b.slots, 0u,
                       b.rpk, b.h, b.sig_status, b.pk_status, b.f, b.ngroups, b.gsum, b.gpair, b.groups, b.upk, b.npk,
                       static_cast<const g1_jac*>(b.gpk), b.gpkp);
  else if (b.ngroups <= bgv_latency_max())
    launch_miller_latency(b, 0u, b.ngroups, st);
  else
    hipLaunchKernelGGL(k_gpair, dim3(nblk(b.ngroups, 64)), dim3(64), 0, st, b.ngroups, b.gsum, b.gpair);
  return hipGetLastError();
}
