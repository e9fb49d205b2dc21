// Group closing kernels (gfx950): team-parallel products and the final exponentiation
// check (bls_team.h), and the Fp12 partial products exchanged across processes
// (per-GPU Miller-loop products gathered for one final exponentiation).
#include "bgv_device.h"

#include "bgv_team_dev.h"
#include "bgv_rns.h"


// A group's verdict bits from its u (bls_team.h tm_final_exp_u; pairing value conj(u)/u):
// bit 0: the pairing value is 1 (u in Fp6).  bit 1 (gu1 given: a retry round with pattern
// tests): it equals the value of the first-pass group ref1 - 1, i.e. u_ref conj(u) lies in
// Fp6 -- the rest of that group, whose value is the quotient, passes.  gu1 is uniform over
// the grid, so every lane of a block takes the same branch and reaches the same barriers.
template <class O>
__device__ int32_t verdict_bits(O& o, const fp_t& u, const bgv_dgroup& g, const fp12_t* __restrict__ gu1, int fi) {
  int32_t v = o.is_fp6(u) ? 1 : 0;
  if (gu1) {
    const fp_t ur = g.ref1 ? reinterpret_cast<const fp_t*>(gu1 + (g.ref1 - 1))[fi] : u;
    if (o.is_fp6(o.mul(ur, o.conj(u))) && g.ref1) v |= 2;
  }
  return v;
}

extern "C" {

// One team per device group (first pass: the groups of the layout; retry rounds: parts of
// failed groups), each a contiguous range of <= 64 slots: v = prod f_i * g_g with
// coefficient-parallel team products (operands straight from the per-slot array), then
// the final-exponentiation check v^((p^12-1)/r) == 1.  The teams of a wave loop to the
// wave's longest group, the shorter ones multiplying by 1, so every lane reaches every
// barrier.
__global__ void BGV_KATTR k_final(const bgv_dgroup* __restrict__ groups, uint32_t ngroups,
                                  const fp12_t* __restrict__ f, const fp12_t* __restrict__ gpair,
                                  int32_t* __restrict__ verdict, fp12_t* __restrict__ gprod,
                                  fp12_t* __restrict__ gu, const fp12_t* __restrict__ gu1) {
  __shared__ fp_t lds[BGV_FINAL_TEAMS][2 * BGV_TEAM_COMPS];
  __shared__ uint32_t lens[BGV_FINAL_TEAMS];
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const int cc = c < BGV_TEAM_COMPS ? c : c - 4;
  const uint32_t gi = blockIdx.x * BGV_FINAL_TEAMS + team;
  // teams past the end duplicate the last group
  const uint32_t gg = gi < ngroups ? gi : ngroups - 1;
  const bgv_dgroup g = groups[gg];
  if (c == 0) lens[team] = g.n_slots;
  __syncthreads();
  uint32_t nmax = 0;
  BGV_UNROLL for (int t = 0; t < BGV_FINAL_TEAMS; ++t) nmax = lens[t] > nmax ? lens[t] : nmax;
  const int fi = tm_fp_index(cc);
  const fp_t one_c = cc == 0 ? fp_one() : fp_zero();  // component cc of 1
  tm_dev_ops o{lds[team], lds[team] + BGV_TEAM_COMPS, c, cc};
  const fp_t* fs = reinterpret_cast<const fp_t*>(f + g.first_slot);
  constexpr int kFp12 = (int)(sizeof(fp12_t) / sizeof(fp_t));
  // the group's signature pair first, then its slots
  fp_t x = reinterpret_cast<const fp_t*>(gpair + gg)[fi];
  fp_t y = grp_has(g, 0) ? fs[fi] : one_c;
  BGV_NO_UNROLL for (uint32_t k = 0; k < nmax; ++k) {
    // next operand in flight (1 for a slot outside the group's mask)
    const fp_t yn = grp_has(g, k + 1) ? fs[kFp12 * (k + 1) + fi] : one_c;
    x = o.mul(x, y);
    y = yn;
  }
  // the group's Miller-loop product, kept for cross-process partials (bgv_verify_partial)
  if (gprod && gi < ngroups && c < BGV_TEAM_COMPS) reinterpret_cast<fp_t*>(gprod + gi)[fi] = x;
  const fp_t u = tm_final_exp_u(o, x);
  if (gu && gi < ngroups && c < BGV_TEAM_COMPS) reinterpret_cast<fp_t*>(gu + gi)[fi] = u;
  const int32_t v = verdict_bits(o, u, g, gu1, fi);
  if (gi < ngroups && c == 0) verdict[gi] = v;
}

// k_final on teams of 12 lanes, five per wave (lanes 60..63 run a sixth, idle team on LDS
// slots of their own so every lane reaches every barrier): a fifth fewer waves for the
// same groups.  Same products in the same order as k_final, so the same verdicts.
// gpkp (nullable; first passes with uniform groups): a BGV_GROUP_UNIFORM group multiplies its
// one pubkey-sum pair gpkp[g] instead of its slots' own pairs.
#define BGV_FINAL12_TEAMS 5
#define BGV_FINAL12_ARGS                                                                                     \
  const bgv_dgroup *__restrict__ groups, uint32_t ngroups, const fp12_t *__restrict__ f,                     \
      const fp12_t *__restrict__ gpair, int32_t *__restrict__ verdict, fp12_t *__restrict__ gprod,          \
      fp12_t *__restrict__ gu, const fp12_t *__restrict__ gu1, const fp12_t *__restrict__ gpkp
}  // extern "C"
__device__ __forceinline__ void final12_body(BGV_FINAL12_ARGS) {
  __shared__ fp_t lds[BGV_FINAL12_TEAMS + 1][2 * BGV_TEAM_COMPS];
  __shared__ uint32_t lens[BGV_FINAL12_TEAMS + 1];
  const int team = threadIdx.x / BGV_TEAM_COMPS, c = threadIdx.x % BGV_TEAM_COMPS;
  const uint32_t gi = blockIdx.x * BGV_FINAL12_TEAMS + team;
  const bool live = team < BGV_FINAL12_TEAMS && gi < ngroups;
  // teams past the end (and the idle sixth) read the last group and multiply by 1
  const bgv_dgroup g = groups[live ? gi : ngroups - 1];
  // the group's slots (<= 64, bgv_launch_groups) as a bit set: the product runs over the
  // present ones only (a retry test masks half of a group or a single job), the teams of the
  // wave to the longest list, multiplying by 1 past their own
  uint64_t m = live ? g.mask & (g.n_slots >= 64 ? ~0ull : ((1ull << g.n_slots) - 1)) : 0;
  const bool uni = gpkp && live && (g.flags & BGV_GROUP_UNIFORM);
  if (uni) m = 0;  // its slots' pairs are the one pair gpkp[gi]
  if (c == 0) lens[team] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t nmax = 0;
  BGV_UNROLL for (int t = 0; t <= BGV_FINAL12_TEAMS; ++t) nmax = lens[t] > nmax ? lens[t] : nmax;
  const int fi = tm_fp_index(c);
  const fp_t one_c = c == 0 ? fp_one() : fp_zero();
  tm_dev_ops_t<BGV_TEAM_COMPS> o{lds[team], lds[team] + BGV_TEAM_COMPS, c, c};
  const fp_t* fs = reinterpret_cast<const fp_t*>(f + g.first_slot);
  constexpr int kFp12 = (int)(sizeof(fp12_t) / sizeof(fp_t));
  fp_t x = reinterpret_cast<const fp_t*>(gpair + (live ? gi : ngroups - 1))[fi];
  auto next = [&]() {  // the next present slot's coefficient, or 1
    if (!m) return one_c;
    const int k = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    return fs[kFp12 * k + fi];
  };
  fp_t y = next();
  BGV_NO_UNROLL for (uint32_t k = 0; k < nmax; ++k) {
    const fp_t yn = next();  // next operand in flight
    x = o.mul(x, y);
    y = yn;
  }
  if (gpkp) x = o.mul(x, uni ? reinterpret_cast<const fp_t*>(gpkp + gi)[fi] : one_c);  // grid-uniform branch
  if (gprod && live) reinterpret_cast<fp_t*>(gprod + gi)[fi] = x;
  const fp_t u = tm_final_exp_u(o, x);
  if (gu && live) reinterpret_cast<fp_t*>(gu + gi)[fi] = u;
  const int32_t v = verdict_bits(o, u, g, gu1, fi);
  if (live && c == 0) verdict[gi] = v;
}

// Weighted tests (BGV_GROUP_WEIGHTED) after k_final12 of a retry round: the first w <= n_slots
// with V^w = W, V the value of first-pass group ref1 - 1 and W the test's (values conj(u) / u:
// u_ref^w conj(u) in Fp6), into verdict bits 8..15 (0: none).  Teams of 12 lanes as k_final12;
// every team of a block runs to the block's longest group (the barriers inside o.mul).
extern "C" __global__ void __launch_bounds__(64) k_final_wident(const bgv_dgroup* __restrict__ groups, uint32_t ngroups,
                                                     const fp12_t* __restrict__ gu, const fp12_t* __restrict__ gu1,
                                                     int32_t* __restrict__ verdict) {
  __shared__ fp_t lds[BGV_FINAL12_TEAMS + 1][2 * BGV_TEAM_COMPS];
  __shared__ uint32_t lens[BGV_FINAL12_TEAMS + 1];
  const int team = threadIdx.x / BGV_TEAM_COMPS, c = threadIdx.x % BGV_TEAM_COMPS;
  const uint32_t gi = blockIdx.x * BGV_FINAL12_TEAMS + team;
  const bool live = team < BGV_FINAL12_TEAMS && gi < ngroups;
  const bgv_dgroup g = groups[live ? gi : ngroups - 1];
  const bool wt = live && (g.flags & BGV_GROUP_WEIGHTED) && g.ref1;
  if (c == 0) lens[team] = wt ? g.n_slots : 0u;
  if (!__syncthreads_or(wt ? 1 : 0)) return;  // the whole block: no weighted test
  uint32_t wmax = 0;
  BGV_UNROLL for (int t = 0; t <= BGV_FINAL12_TEAMS; ++t) wmax = lens[t] > wmax ? lens[t] : wmax;
  const int fi = tm_fp_index(c);
  const fp_t one_c = c == 0 ? fp_one() : fp_zero();
  tm_dev_ops_t<BGV_TEAM_COMPS> o{lds[team], lds[team] + BGV_TEAM_COMPS, c, c};
  const fp_t u = wt ? reinterpret_cast<const fp_t*>(gu + gi)[fi] : one_c;
  const fp_t ur = wt ? reinterpret_cast<const fp_t*>(gu1 + (g.ref1 - 1))[fi] : one_c;
  const fp_t cu = o.conj(u);
  fp_t P = ur;
  int32_t found = 0;
  BGV_NO_UNROLL for (uint32_t w = 1; w <= wmax; ++w) {
    const bool hit = o.is_fp6(o.mul(P, cu));
    if (wt && hit && found == 0 && w <= g.n_slots) found = (int32_t)w;
    P = o.mul(P, ur);
  }
  if (wt && c == 0) verdict[gi] = (verdict[gi] & 1) | (found << 8);
}
extern "C" {
// Two waves per SIMD: the same 250 VGPRs and 128 B of scratch per lane as at one, and the teams'
// barrier and LDS waits overlap the other wave's products: headline 2.457-2.461 vs 2.425-2.427 M
// sets/s, interleaved (profiles/r05/retry_variants/ab_w2.jsonl, ab_base.jsonl)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) k_final12(BGV_FINAL12_ARGS) {
  final12_body(groups, ngroups, f, gpair, verdict, gprod, gu, gu1, gpkp);
}

// The latency path's closing (small calls): one block of BGV_FOLD_TEAMS (16) teams per group.
// Team t multiplies the group's slots t, t + 16, ... (team 0 also the signature pair), the
// partial products meet in LDS in a four-level tree (a sixteenth of k_final's serial product
// chain; 8 teams measured 0.86 ms for the 64-set gossip call).  The final exponentiation then runs on the
// whole block with each coefficient's products split over eight lanes (tm_wide_ops_t<false, 8>):
// one double-width product per lane for a squaring (two for a product) instead of 7 on one.
// ENGINE 2 (round 6, the default k_final_fold): the final exponentiation in residue arithmetic
// (bgv_rns.h) on a 384-thread block, one residue of one coefficient per lane and one Montgomery
// reduction (two base extensions) per coefficient and operation: 0.96 against 1.89 us per Fp12
// operation of the eight-part engine (tools/ubench_rns.hip, profiles/r06/rns/); the fold keeps
// its 16 teams, the block's other 128 threads (teams 16..23) run the same products on ones so
// every thread reaches every barrier.  ENGINE 1 (k_final_fold_p8, BGV_FOLD_RNS=0): the
// eight-part engine with the lane's squaring recipes (bgv_team_dev.h tm_wide8_lean_ops);
// ENGINE 0 (k_final_fold_sel, BGV_FOLD_RNS=0 BGV_FOLD_LEAN=0) its select-based forms.  The same
// field elements every way: u, the verdict bits and gu agree.
}  // extern "C"
template <bool LEAN>
__device__ auto bgv_fold_ops_pick() {
  if constexpr (LEAN)
    return tm_wide8_lean_ops{};
  else
    return tm_wide_ops_t<false, 8>{};
}
#ifndef BGV_FOLD_TEAMS
#define BGV_FOLD_TEAMS 16  // 16-lane teams of k_final_fold's fold (BGV_FOLD_THREADS threads)
#endif
#define BGV_FOLD_THREADS (BGV_FOLD_TEAMS * BGV_TEAM)
#define BGV_FOLD_RNS_THREADS BGV_RNS_THREADS
static_assert(BGV_FOLD_RNS_THREADS % BGV_TEAM == 0 && BGV_FOLD_RNS_THREADS >= BGV_FOLD_THREADS, "fold block");
template <int ENGINE>
__device__ __forceinline__ void final_fold_body(const bgv_dgroup* __restrict__ groups, uint32_t ngroups,
                                                const fp12_t* __restrict__ f, const fp12_t* __restrict__ gpair,
                                                int32_t* __restrict__ verdict, fp12_t* __restrict__ gprod,
                                                fp12_t* __restrict__ gu, const fp12_t* __restrict__ gu1,
                                                const fp12_t* __restrict__ fsig, const fp12_t* __restrict__ gpkp) {
  constexpr int kTeams = (ENGINE == 2 ? BGV_FOLD_RNS_THREADS : BGV_FOLD_THREADS) / BGV_TEAM;
  __shared__ fp_t lds[kTeams][2 * BGV_TEAM_COMPS];
  __shared__ fp_t part[BGV_FOLD_TEAMS][BGV_TEAM_COMPS];
  __shared__ fp_t W[BGV_TEAM_COMPS], WA[BGV_TEAM_COMPS], WB[BGV_TEAM_COMPS], WP[8 * BGV_TEAM_COMPS];
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const bool fold = team < BGV_FOLD_TEAMS;  // teams past the fold's 16 multiply ones
  const int cc = c < BGV_TEAM_COMPS ? c : c - 4;
  const uint32_t gi = blockIdx.x;
  const bgv_dgroup g = groups[gi < ngroups ? gi : ngroups - 1];
  const int fi = tm_fp_index(cc);
  const fp_t one_c = cc == 0 ? fp_one() : fp_zero();
  tm_dev_ops o{lds[team], lds[team] + BGV_TEAM_COMPS, c, cc};
  const fp_t* fs = reinterpret_cast<const fp_t*>(f + g.first_slot);
  constexpr int kFp12 = (int)(sizeof(fp12_t) / sizeof(fp_t));
  // the group's signature pair, or (fsig: bgv_sig_pairs) each slot's own
  fp_t x = team == 0 && !fsig ? reinterpret_cast<const fp_t*>(gpair + (gi < ngroups ? gi : ngroups - 1))[fi] : one_c;
  const fp_t* ss = fsig ? reinterpret_cast<const fp_t*>(fsig + g.first_slot) : nullptr;
  // gpkp (retry rounds of uniform batches, as k_final12): a uniform test multiplies its one
  // pubkey-sum pair instead of its slots' pairs (uniform over the block)
  const bool uni = gpkp && gi < ngroups && (g.flags & BGV_GROUP_UNIFORM);
  const uint32_t nmax = uni ? 0u : (g.n_slots + BGV_FOLD_TEAMS - 1) / BGV_FOLD_TEAMS;
  BGV_NO_UNROLL for (uint32_t k = 0; k < nmax; ++k) {
    const uint32_t idx = team + BGV_FOLD_TEAMS * k;
    const bool in = fold && grp_has(g, idx);
    const fp_t y = in ? fs[kFp12 * idx + fi] : one_c;
    x = o.mul(x, y);
    if (ss) x = o.mul(x, in ? ss[kFp12 * idx + fi] : one_c);  // grid-uniform branch
  }
  // the eight partial products as a tree: every team multiplies at every level (the barriers
  // inside o.mul), team t keeps parts 2t and 2t + 1 of the level
  BGV_UNROLL for (int w = BGV_FOLD_TEAMS; w > 1; w >>= 1) {
    if (fold && c < BGV_TEAM_COMPS) part[team][cc] = x;
    __syncthreads();
    const int t2 = 2 * (team % (w >> 1));
    x = o.mul(part[t2][cc], part[t2 + 1][cc]);
  }
  if (gpkp) x = o.mul(x, uni && team == 0 ? reinterpret_cast<const fp_t*>(gpkp + gi)[fi] : one_c);  // grid-uniform
  if (gprod && gi < ngroups && team == 0 && c < BGV_TEAM_COMPS) reinterpret_cast<fp_t*>(gprod + gi)[fi] = x;
  // the final exponentiation on the whole block with the wide products (bgv_team_dev.h)
  if (team == 0 && c < BGV_TEAM_COMPS) W[cc] = x;
  __syncthreads();
  if constexpr (ENGINE == 2) {
    // residue arithmetic (bgv_rns.h): W in, u (and gu, the verdict bits) out; every branch
    // below is uniform over the block (gu, gu1 over the grid, g.ref1 over the block)
    __shared__ rns_smem RS;
    rns_ops ro;
    ro.init(&RS, threadIdx.x);
    const uint32_t u = tm_final_exp_u(ro, ro.from_fp(W[ro.c]));
    const int rfi = tm_fp_index(ro.c);
    if (gu && gi < ngroups) {
      const fp_t uf = ro.to_fp(u);
      if (ro.i == 0) reinterpret_cast<fp_t*>(gu + gi)[rfi] = uf;
    }
    int32_t v = ro.is_fp6(u) ? 1 : 0;
    if (gu1 && g.ref1) {  // see verdict_bits
      const uint32_t ur = ro.from_fp(reinterpret_cast<const fp_t*>(gu1 + (g.ref1 - 1))[rfi]);
      if (ro.is_fp6(ro.mul(ur, ro.conj(u)))) v |= 2;
    }
    if (gi < ngroups && threadIdx.x == 0) verdict[gi] = v;
  } else {
    const int wc = threadIdx.x % BGV_TEAM_COMPS, wq = threadIdx.x / BGV_TEAM_COMPS;
    using OW = decltype(bgv_fold_ops_pick<ENGINE == 1>());
    OW ow;
    ow.A = WA;
    ow.B = WB;
    ow.P = WP;
    ow.c = wc;
    ow.q = wq;
    if constexpr (ENGINE == 1) tm_sqr_rec8(wc, wq, &ow.rx, &ow.ry);
    const fp_t xw = W[wc];
    const int wfi = tm_fp_index(wc);
    const fp_t u = tm_final_exp_u(ow, xw);
    if (gu && gi < ngroups && wq == 0) reinterpret_cast<fp_t*>(gu + gi)[wfi] = u;
    const int32_t v = verdict_bits(ow, u, g, gu1, wfi);
    if (gi < ngroups && threadIdx.x == 0) verdict[gi] = v;
  }
}
extern "C" {
#define BGV_FOLD_ARGS                                                                                         \
  const bgv_dgroup *__restrict__ groups, uint32_t ngroups, const fp12_t *__restrict__ f,                     \
      const fp12_t *__restrict__ gpair, int32_t *__restrict__ verdict, fp12_t *__restrict__ gprod,          \
      fp12_t *__restrict__ gu, const fp12_t *__restrict__ gu1, const fp12_t *__restrict__ fsig,                \
      const fp12_t *__restrict__ gpkp
__global__ void __launch_bounds__(BGV_FOLD_RNS_THREADS) k_final_fold(BGV_FOLD_ARGS) {
  final_fold_body<2>(groups, ngroups, f, gpair, verdict, gprod, gu, gu1, fsig, gpkp);
}
__global__ void __launch_bounds__(BGV_FOLD_THREADS) k_final_fold_p8(BGV_FOLD_ARGS) {
  final_fold_body<1>(groups, ngroups, f, gpair, verdict, gprod, gu, gu1, fsig, gpkp);
}
__global__ void __launch_bounds__(BGV_FOLD_THREADS) k_final_fold_sel(BGV_FOLD_ARGS) {
  final_fold_body<0>(groups, ngroups, f, gpair, verdict, gprod, gu, gu1, fsig, gpkp);
}

// Products of runs of Fp12 values (cross-process partials): team t of the
// grid multiplies in[t * chunk, min(n, (t + 1) * chunk)) into out[t] (1 for an empty run).
// Teams of a wave loop to the wave's longest run, multiplying by 1, so every lane reaches
// every barrier.
__global__ void BGV_KATTR k_fp12_prod(const fp12_t* __restrict__ in, uint32_t n, uint32_t chunk,
                                      fp12_t* __restrict__ out, uint32_t nout) {
  __shared__ fp_t lds[BGV_FINAL_TEAMS][2 * BGV_TEAM_COMPS];
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const int cc = c < BGV_TEAM_COMPS ? c : c - 4;
  const uint32_t t = blockIdx.x * BGV_FINAL_TEAMS + team;
  const uint32_t lo = t * chunk;
  const uint32_t len = lo < n ? (n - lo < chunk ? n - lo : chunk) : 0;
  const int fi = tm_fp_index(cc);
  const fp_t one_c = cc == 0 ? fp_one() : fp_zero();
  tm_dev_ops o{lds[team], lds[team] + BGV_TEAM_COMPS, c, cc};
  fp_t x = one_c;
  for (uint32_t k = 0; k < chunk; ++k) {  // chunk is uniform: every team runs chunk products
    const fp_t y = k < len ? reinterpret_cast<const fp_t*>(in + lo + k)[fi] : one_c;
    x = o.mul(x, y);
  }
  if (t < nout && c < BGV_TEAM_COMPS) reinterpret_cast<fp_t*>(out + t)[fi] = x;
}

// Fp12 <-> 576 canonical big-endian bytes: the 12 Fp coefficients in tower order
// (c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1), 48 bytes each.
__global__ void k_fp12_to_bytes(const fp12_t* __restrict__ in, uint8_t* __restrict__ out576) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const fp_t* v = reinterpret_cast<const fp_t*>(in);
  for (int i = 0; i < 12; ++i) {
    uint8_t b[48];
    fp_to_be48(b, fp_from_mont(v[i]));
    for (int q = 0; q < 48; ++q) out576[48 * i + q] = b[q];
  }
}

// n values -> 576 canonical bytes each (one lane per value; parity hooks)
__global__ void k_fp12_n_to_bytes(const fp12_t* __restrict__ in, uint32_t n, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fp_t* v = reinterpret_cast<const fp_t*>(in + i);
  for (int k = 0; k < 12; ++k) {
    uint8_t b[48];
    fp_to_be48(b, fp_from_mont(v[k]));
    for (int q = 0; q < 48; ++q) out[576ull * i + 48 * k + q] = b[q];
  }
}

// n serialized values -> Montgomery Fp12; status[i] = 0, or BGV_BAD_ENCODING for a
// coefficient >= p.  one[0] receives 1 (the group pair slot of a k_final over the values).
__global__ void k_fp12_from_bytes(const uint8_t* __restrict__ in, uint32_t n, fp12_t* __restrict__ out,
                                  int32_t* __restrict__ status, fp12_t* __restrict__ one) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *one = fp12_one();
  if (i >= n) return;
  fp_t* v = reinterpret_cast<fp_t*>(out + i);
  int32_t st = BGV_OK;
  for (int k = 0; k < 12; ++k) {
    uint8_t b[48];
    for (int q = 0; q < 48; ++q) b[q] = in[576ull * i + 48 * k + q];
    const fp_t r = fp_from_be48(b);
    if (!fp_raw_lt_p(r)) st = BGV_BAD_ENCODING;
    v[k] = fp_to_mont(r);
  }
  status[i] = st;
}

}  // extern "C"

// Group closing over b.groups (contiguous slot ranges of <= 64 slots) after
// bgv_launch_miller (first pass, group pairs already made) or, for a retry round over the
// same per-slot results, with pairs = true: the parts' signature sums and pairs first.
uint32_t bgv_fold_pairs_max() { return bgv_latency_max(); }
#ifndef BGV_RETRY_FOLD_MAX
#define BGV_RETRY_FOLD_MAX 512
#endif

hipError_t bgv_launch_groups(const bgv_dev_batch& b, const bgv_streams& s, bool pairs) {
  if (b.ngroups == 0) return hipSuccess;
  BGV_MARK(4);
  if (pairs) {
    const hipError_t e = bgv_launch_gpairs(b, s.main);
    if (e != hipSuccess) return e;
  }
  static const bool lean = [] {
    const char* e = getenv("BGV_FOLD_LEAN");
    return !(e && atoi(e) == 0);
  }();
  static const bool rns = [] {
    const char* e = getenv("BGV_FOLD_RNS");
    return !(e && atoi(e) == 0);
  }();
  if (b.weighted && !b.gu) return hipErrorInvalidValue;
  // A retry round of a uniform batch (b.uniform: tests inside uniform first-pass groups, whose
  // slots have no pair f_i of their own) closes on k_final12, which multiplies the tests' pubkey-
  // sum pairs (gpkp), whatever its size: its b.ngroups counts only the round's tests, so a batch
  // just above the latency bound on its first pass can fall below it here (advisor r05), and
  // k_final_fold would multiply the groups' unwritten f_i instead.
  // A retry round of a uniform batch with at most BGV_RETRY_FOLD_MAX tests (env; 0: none)
  // closes on k_final_fold whatever the batch's size: one block per test, its final
  // exponentiation in residue arithmetic (~0.55 against ~2.8 ms for k_final12's teams) at ~6x
  // the SIMD time per test.  Mainnet-shaped windows (uniform batches, their rate bound by the
  // retry thread's round latency): 5.05-5.17 against 4.47-4.81 M sets/s; on the headline's
  // non-uniform batches it cost 0.4 % (512 tests) to 30 % (every round), so those stay on
  // k_final12 (profiles/r06/retry_fold/).
  static const uint32_t retry_fold_max = [] {
    const char* e = getenv("BGV_RETRY_FOLD_MAX");
    return e ? (uint32_t)atoi(e) : (uint32_t)BGV_RETRY_FOLD_MAX;
  }();
  const bool small_retry = pairs && b.uniform && b.ngroups <= retry_fold_max;
  if ((!b.uniform && b.nslots + b.ngroups <= bgv_latency_max()) || small_retry)
    hipLaunchKernelGGL(rns ? k_final_fold : (lean ? k_final_fold_p8 : k_final_fold_sel), dim3(b.ngroups),
                       dim3(rns ? BGV_FOLD_RNS_THREADS : BGV_FOLD_THREADS), 0, s.main, b.groups,
                       b.ngroups, b.f, b.gpair,
                       b.verdict, b.gprod, b.gu, b.gu1,
                       !pairs && bgv_sig_pairs(b) ? static_cast<const fp12_t*>(b.fsig) : nullptr,
                       b.uniform ? static_cast<const fp12_t*>(b.gpkp) : nullptr);
  else
    hipLaunchKernelGGL(k_final12, dim3(nblk(b.ngroups, BGV_FINAL12_TEAMS)), dim3(64), 0, s.main, b.groups,
                       b.ngroups, b.f, b.gpair, b.verdict, b.gprod, b.gu, b.gu1,
                       b.uniform ? static_cast<const fp12_t*>(b.gpkp) : nullptr);
  if (b.weighted)
    hipLaunchKernelGGL(k_final_wident, dim3(nblk(b.ngroups, BGV_FINAL12_TEAMS)), dim3(64), 0, s.main, b.groups,
                       b.ngroups, static_cast<const fp12_t*>(b.gu), b.gu1, b.verdict);
  BGV_MARK(5);
  return hipGetLastError();
}
// Product of groups [g0, g0 + ng) of the last k_final (b.gprod) -> 576 canonical bytes.
// scratch: (ng / 32 + 2) Fp12 values.
hipError_t bgv_launch_partial(const bgv_dev_batch& b, uint32_t g0, uint32_t ng, void* scratch, uint8_t* out576,
                              hipStream_t st) {
  fp12_t* tmp = reinterpret_cast<fp12_t*>(scratch);
  const uint32_t chunk = 32, n1 = (ng + chunk - 1) / chunk;
  hipLaunchKernelGGL(k_fp12_prod, dim3(nblk(n1 ? n1 : 1, BGV_FINAL_TEAMS)), dim3(64), 0, st, b.gprod + g0, ng, chunk,
                     tmp + 1, n1);
  hipLaunchKernelGGL(k_fp12_prod, dim3(1), dim3(64), 0, st, tmp + 1, n1, n1 ? n1 : 1, tmp, 1u);
  hipLaunchKernelGGL(k_fp12_to_bytes, dim3(1), dim3(64), 0, st, tmp, out576);
  return hipGetLastError();
}
size_t bgv_fp12_bytes() { return sizeof(fp12_t); }
hipError_t bgv_launch_fp12_bytes(const fp12_t* in, uint32_t n, uint8_t* out576, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fp12_n_to_bytes, dim3(nblk(n, 64)), dim3(64), 0, st, in, n, out576);
  return hipGetLastError();
}

// prod of n serialized partials, then the final-exponentiation check (one k_final group)
hipError_t bgv_launch_final_verify(const uint8_t* in, uint32_t n, void* vals, void* one, const bgv_dgroup* group,
                                   int32_t* status, int32_t* verdict, hipStream_t st) {
  hipLaunchKernelGGL(k_fp12_from_bytes, dim3(nblk(n, 64)), dim3(64), 0, st, in, n, reinterpret_cast<fp12_t*>(vals),
                     status, reinterpret_cast<fp12_t*>(one));
  hipLaunchKernelGGL(k_final, dim3(1), dim3(64), 0, st, group, 1u, reinterpret_cast<const fp12_t*>(vals),
                     reinterpret_cast<const fp12_t*>(one), verdict, static_cast<fp12_t*>(nullptr),
                     static_cast<fp12_t*>(nullptr), static_cast<const fp12_t*>(nullptr));
  return hipGetLastError();
}
