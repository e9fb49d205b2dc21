// Batch BLS12-381 signature-set verification kernels for CDNA4 (gfx950).
//
// One signature set per lane.  A verify call runs these kernels in order (see
// bgv_api.cpp):
//
//   k_pk_agg   (only when a call holds a set with >= BGV_PK_TREE_MIN cached keys) one
//              wavefront per such set sums its keys with a ds_swizzle/ds_bpermute tree
//   k_prep     three independent tasks side by side (blockIdx.y):
//              sig  decompress + subgroup-check the 96-byte signature, then r_i * sig_i
//                   (Jacobian G2, summed per group by the closing)
//              hash hash_to_G2(signing root) -> H(m_i), Jacobian
//              pk   gather + aggregate pubkeys from the device cache; r_i * pk_i, affine
//   k_gsum     per device group (a team of 16 lanes): S_g = sum of the group's r_i sig_i
//   k_miller   f_i = MillerLoop(r_i pk_i, H(m_i)), one pair per lane, and on extra lanes
//              one per group g_g = MillerLoop(-G1, S_g) (retry rounds: k_gpair)
//   k_final    per device group (a team of 16 lanes): prod f_i * g_g and the
//              final-exponentiation check -> == 1
//
// This is the randomized batch equation of blst's verifyMultipleAggregateSignatures
// (called from packages/beacon-node/src/chain/bls/maybeBatch.ts:18-25):
//   prod_i e(r_i pk_i, H(m_i)) * e(-G1, sum_i r_i sig_i) == 1,
// with blst's structure: one pair per set, r_i sig_i in G2, one signature pair per
// group.  A one-set group is the core verify of maybeBatch.ts:34-38 raised to the
// power r (nonzero, < group order), which has the same verdict.
#include "bgv_layout.h"
#define BGV_KERNEL_SIDE 1
#include "bls_hash.h"
#include "bls_pairing.h"
#include "bls_team.h"

// Waves per SIMD the verify kernels are register-budgeted for (1: up to 512 VGPRs).
#ifndef BGV_WPE
#define BGV_WPE 1
#endif
// k_prep runs 3 x nslots lanes of shorter tasks: two waves per SIMD measured faster
// (36.6 vs 45.3 ms per 131072 slots), the long-chain kernels stay at one.
#ifndef BGV_WPE_PREP
#define BGV_WPE_PREP 2
#endif
// Sets with at least this many cached pubkeys are aggregated by k_pk_agg's wavefront
// tree instead of serially on the set's k_prep lane.
#ifndef BGV_PK_TREE_MIN
#define BGV_PK_TREE_MIN 16
#endif
#define BGV_KATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE, BGV_WPE)))
#define BGV_KATTR_PREP __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE_PREP, BGV_WPE_PREP)))

// Wavefront exchange of one 32-bit word with lane (l ^ m): ds_swizzle in bit-mask mode
// within each 32-lane half (m < 32), ds_bpermute across the halves (m = 32).  No LDS
// storage is allocated: both go through the LDS crossbar only.
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
  if constexpr (M == 32)
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((threadIdx.x ^ 32u) << 2), (int)v);
  else
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1f | (M << 10));  // and 0x1f, xor M
}

template <int M, class P>
__device__ __forceinline__ P point_xor(const P& p) {
  constexpr int W = (int)(sizeof(P) / 4);
  P r;
  const uint32_t* a = reinterpret_cast<const uint32_t*>(&p);
  uint32_t* o = reinterpret_cast<uint32_t*>(&r);
  BGV_UNROLL for (int i = 0; i < W; ++i) o[i] = lane_xor<M>(a[i]);
  return r;
}


extern "C" {

// r_i * sig_i of a set whose signature decodes and lies in G2 (else only a status).
__device__ __noinline__ void task_sig(uint32_t s, const bgv_dslot* __restrict__ slots, g2_jac* __restrict__ rsig,
                                      int32_t* __restrict__ sig_status) {
  const bgv_dslot& d = slots[s];
  int32_t st = BGV_ST_OK;
  if (d.flags & BGV_SLOT_PAD) {
    st = BGV_ST_INFINITY;
  } else if (d.sig_len != 96) {
    st = BGV_INVALID_SIZE;
  } else {
    uint8_t b[96];
    for (int i = 0; i < 96; ++i) b[i] = d.sig[i];
    g2_aff a;
    bool inf;
    st = g2_decompress(&a, &inf, b);
    if (st == BGV_OK) {
      if (inf) {
        st = BGV_ST_INFINITY;  // skipped in the accumulator, as blst does
      } else {
        const g2_jac j = jac_from_aff(a);
        if (!g2_in_subgroup(j))
          st = BGV_POINT_NOT_IN_GROUP;
        else
          rsig[s] = jac_mul_u64(j, d.scalar);  // never infinity: 0 < r < group order
      }
    }
  }
  sig_status[s] = st;
}

__device__ __noinline__ void task_hash(uint32_t s, const bgv_dslot* __restrict__ slots, g2_jac* __restrict__ h) {
  const bgv_dslot& d = slots[s];
  if (d.flags & BGV_SLOT_PAD) return;
  uint8_t msg[32];
  for (int i = 0; i < 32; ++i) msg[i] = d.msg[i];
  h[s] = hash_to_g2(msg, 32);  // stays Jacobian: k_miller adds it with miller_add_jq
}

// Sum of one set's pubkeys (PublicKey.aggregate, chain/bls/utils.ts:5-16): the k_pk_agg
// tree sum when the set went through it, else serial mixed additions of cached keys or of
// 96-byte records (decoded like blst's PublicKey.fromBytes, bls_curve.h g1_deserialize).
// *st receives the first record's decode error, if any.
__device__ __noinline__ static g1_jac pk_sum(const bgv_dslot& d, const uint32_t* __restrict__ pk_idx,
                                      const g1_aff* __restrict__ cache, const uint8_t* __restrict__ pk_bytes,
                                      const g1_jac* __restrict__ pk_agg, uint32_t s, int32_t* st) {
  g1_jac acc = jac_infinity<fp_t>();
  const bool cached = (d.flags & BGV_SLOT_PK_CACHED) != 0;
  const bool tree = pk_agg != nullptr && cached && d.n_pk >= BGV_PK_TREE_MIN;  // summed by k_pk_agg
  if (tree) return pk_agg[s];
  for (uint32_t k = 0; k < d.n_pk; ++k) {
    g1_aff a;
    if (cached) {
      a = cache[pk_idx[d.pk_off + k]];
    } else {
      uint8_t b[96];
      const uint8_t* src = pk_bytes + 96ull * (d.pk_off + k);
      for (int i = 0; i < 96; ++i) b[i] = src[i];
      bool inf;
      const int rc = g1_deserialize(&a, &inf, b);
      if (rc != BGV_OK) {
        *st = rc;
        break;
      }
      if (inf) continue;
    }
    acc = jac_add_aff(acc, a);
  }
  return acc;
}

__device__ __noinline__ void task_pk(uint32_t s, const bgv_dslot* __restrict__ slots,
                                     const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                     const uint8_t* __restrict__ pk_bytes, g1_aff* __restrict__ rpk,
                                     int32_t* __restrict__ pk_status, const g1_jac* __restrict__ pk_agg) {
  const bgv_dslot& d = slots[s];
  int32_t st = BGV_ST_OK;
  if (d.flags & BGV_SLOT_PAD) {
    pk_status[s] = BGV_ST_INFINITY;
    return;
  }
  const g1_jac acc = pk_sum(d, pk_idx, cache, pk_bytes, pk_agg, s, &st);
  if (st == BGV_OK) {
    g1_aff pa;
    if (!jac_to_aff(&pa, jac_mul_u64(acc, d.scalar)))
      st = BGV_ST_INFINITY;  // infinity aggregate: BLST_PK_IS_INFINITY / false (job_precheck)
    else
      rpk[s] = pa;
  }
  pk_status[s] = st;
}

// Pubkey aggregation of many-key sets as a wavefront tree (one wave per slot): lane l
// sums the set's cached keys l, l + 64, ... with mixed additions (coalesced gathers),
// then six butterfly levels of complete Jacobian additions with the partner lane's
// partial sum (lane ^ 32, 16, ..., 1) exchanged in registers.  Every lane ends with the
// total; the sum is the same group element as the serial one.  Waves of slots with fewer
// than BGV_PK_TREE_MIN cached keys exit at once (uniformly: every lane reads the same slot).
__global__ void __launch_bounds__(64) k_pk_agg(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                               const uint32_t* __restrict__ pk_idx,
                                               const g1_aff* __restrict__ cache, g1_jac* __restrict__ pk_agg) {
  const uint32_t s = blockIdx.x;
  if (s >= nslots) return;
  const bgv_dslot& d = slots[s];
  if ((d.flags & BGV_SLOT_PAD) || !(d.flags & BGV_SLOT_PK_CACHED) || d.n_pk < BGV_PK_TREE_MIN) return;
  const uint32_t l = threadIdx.x;
  g1_jac acc = jac_infinity<fp_t>();
  for (uint32_t k = l; k < d.n_pk; k += 64) acc = jac_add_aff(acc, cache[pk_idx[d.pk_off + k]]);
  acc = jac_add(acc, point_xor<32>(acc));
  acc = jac_add(acc, point_xor<16>(acc));
  acc = jac_add(acc, point_xor<8>(acc));
  acc = jac_add(acc, point_xor<4>(acc));
  acc = jac_add(acc, point_xor<2>(acc));
  acc = jac_add(acc, point_xor<1>(acc));
  if (l == 0) pk_agg[s] = acc;
}

// The three independent per-set tasks in one launch (blockIdx.y = task), so one
// batch keeps 3x the wavefronts in flight on a single stream.
__global__ void BGV_KATTR_PREP k_prep(const bgv_dslot* __restrict__ slots, uint32_t nslots, g2_jac* __restrict__ rsig,
                                      int32_t* __restrict__ sig_status, g2_jac* __restrict__ h,
                                      const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                      const uint8_t* __restrict__ pk_bytes, g1_aff* __restrict__ rpk,
                                      int32_t* __restrict__ pk_status, const g1_jac* __restrict__ pk_agg) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  // hash first: the longest task starts earliest
  if (blockIdx.y == 0)
    task_hash(s, slots, h);
  else if (blockIdx.y == 1)
    task_sig(s, slots, rsig, sig_status);
  else
    task_pk(s, slots, pk_idx, cache, pk_bytes, rpk, pk_status, pk_agg);
}

// A slot takes part in its group's equation iff it is a set whose signature decoded
// (valid or infinity) and whose pubkeys aggregated to a finite point; its signature
// joins the group's sum only when it is not the infinity signature (blst skips those).
__device__ __forceinline__ bool slot_live(const bgv_dslot& d, int32_t ss, int32_t ps) {
  return !(d.flags & BGV_SLOT_PAD) && (ss == BGV_ST_OK || ss == BGV_ST_INFINITY) && ps == BGV_ST_OK;
}

// Lanes [0, nslots): f_i = MillerLoop(r pk, H(m)), 1 for slots that do not take part.
// Lanes [nslots, nslots + ngroups): the group's signature pair MillerLoop(-G1, S_g) (1 for
// an infinite S_g), so the group pairs run beside the set pairs instead of after them.
__device__ __forceinline__ fp12_t group_pair(const g2_jac& S) {
  return jac_is_inf(S) ? fp12_one() : miller_loop1(g1_neg_generator(), S);
}

__global__ void BGV_KATTR k_miller(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                   const g1_aff* __restrict__ rpk, const g2_jac* __restrict__ h,
                                   const int32_t* __restrict__ sig_status, const int32_t* __restrict__ pk_status,
                                   fp12_t* __restrict__ f, uint32_t ngroups, const g2_jac* __restrict__ gsum,
                                   fp12_t* __restrict__ gpair) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < nslots) {
    fp12_t r = fp12_one();
    if (slot_live(slots[s], sig_status[s], pk_status[s])) r = miller_loop1(rpk[s], h[s]);
    f[s] = r;
  } else if (s - nslots < ngroups) {
    gpair[s - nslots] = group_pair(gsum[s - nslots]);
  }
}

// retry rounds: the signature pairs of the round's parts alone
__global__ void BGV_KATTR k_gpair(uint32_t ngroups, const g2_jac* __restrict__ gsum, fp12_t* __restrict__ gpair) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ngroups) gpair[g] = group_pair(gsum[g]);
}

// Group closing, team-parallel (bls_team.h): a team of 16 lanes per group, lane c < 12
// owning one Fp coefficient of the running value; operands exchanged through LDS.
__constant__ fp2_t kTeamFrob1[6] = BGV_FROB1;
__constant__ fp_t kTeamFrob2[6] = BGV_FROB2;

struct tm_dev_ops {
  fp_t* A;  // this team's 12 + 12 LDS slots
  fp_t* B;
  int c;   // lane within the team, 0..15
  int cc;  // component computed by this lane (lanes 12..15 duplicate 8..11)
  __device__ fp_t mul(const fp_t& x, const fp_t& y) {
    if (c < BGV_TEAM_COMPS) {
      A[c] = x;
      B[c] = y;
    }
    __syncthreads();
    const fp_t r = tm_mul_lane(cc, A, B);
    __syncthreads();
    return r;
  }
  __device__ fp_t sqr(const fp_t& x) {
    if (c < BGV_TEAM_COMPS) A[c] = x;
    __syncthreads();
    const fp_t r = tm_sqr_lane(cc, A);
    __syncthreads();
    return r;
  }
  __device__ fp_t line(const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) { return tm_line_lane(cc, l0, l1, l3); }
  __device__ fp_t mul_line(const fp_t& x, const fp2_t& l0, const fp2_t& l1, const fp2_t& l3) {
    if (c < BGV_TEAM_COMPS) A[c] = x;
    __syncthreads();
    const fp_t r = tm_mul_line_lane(cc, A, l0, l1, l3);
    __syncthreads();
    return r;
  }
  __device__ fp_t conj(const fp_t& x) { return fp_select(((cc >> 1) & 1) != 0, x, fp_neg(x)); }
  __device__ fp_t frob(const fp_t& x) {
    if (c < BGV_TEAM_COMPS) A[c] = x;
    __syncthreads();
    const fp_t x0 = A[cc & ~1], x1 = A[cc | 1];
    __syncthreads();
    return tm_frob_lane(cc, x0, x1, kTeamFrob1[tm_tower_pos(cc)]);
  }
  __device__ fp_t frob2(const fp_t& x) { return fp_mul(x, kTeamFrob2[tm_tower_pos(cc)]); }
  __device__ bool is_fp6(const fp_t& x) {
    const bool bad = c < BGV_TEAM_COMPS && ((cc >> 1) & 1) && !fp_is_zero(x);
    const uint64_t m = __ballot(bad);
    return ((m >> (threadIdx.x & ~(BGV_TEAM - 1))) & 0xffffu) == 0;
  }
};

#define BGV_FINAL_TEAMS (64 / BGV_TEAM)
// S_g = sum of r_i sig_i over a group's live, non-infinity signatures (blst skips an
// infinity signature in the accumulator).  A team of 16 lanes per group: lane c sums
// every 16th slot, then a 4-level ds_swizzle butterfly; the team leader writes S_g.
__global__ void __launch_bounds__(64) k_gsum(const bgv_dgroup* __restrict__ groups, uint32_t ngroups,
                                             const bgv_dslot* __restrict__ slots, const g2_jac* __restrict__ rsig,
                                             const int32_t* __restrict__ sig_status,
                                             const int32_t* __restrict__ pk_status, g2_jac* __restrict__ gsum) {
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const uint32_t gi = blockIdx.x * BGV_FINAL_TEAMS + team;
  const bgv_dgroup g = groups[gi < ngroups ? gi : ngroups - 1];
  g2_jac acc = jac_infinity<fp2_t>();
  for (uint32_t k = (uint32_t)c; k < g.n_slots; k += BGV_TEAM) {
    const uint32_t s = g.first_slot + k;
    const int32_t ss = sig_status[s];
    if (ss == BGV_ST_OK && slot_live(slots[s], ss, pk_status[s])) acc = jac_add(acc, rsig[s]);
  }
  acc = jac_add(acc, point_xor<8>(acc));
  acc = jac_add(acc, point_xor<4>(acc));
  acc = jac_add(acc, point_xor<2>(acc));
  acc = jac_add(acc, point_xor<1>(acc));
  if (gi < ngroups && c == 0) gsum[gi] = acc;
}

// One team per device group (first pass: the groups of the layout; retry rounds: parts of
// failed groups), each a contiguous range of <= 64 slots: v = prod f_i * g_g with
// coefficient-parallel team products (operands straight from the per-slot array), then
// the final-exponentiation check v^((p^12-1)/r) == 1.  The teams of a wave loop to the
// wave's longest group, the shorter ones multiplying by 1, so every lane reaches every
// barrier.
__global__ void BGV_KATTR k_final(const bgv_dgroup* __restrict__ groups, uint32_t ngroups,
                                  const fp12_t* __restrict__ f, const fp12_t* __restrict__ gpair,
                                  int32_t* __restrict__ verdict) {
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
  fp_t y = g.n_slots ? fs[fi] : one_c;
  BGV_NO_UNROLL for (uint32_t k = 0; k < nmax; ++k) {
    const fp_t yn = k + 1 < g.n_slots ? fs[kFp12 * (k + 1) + fi] : one_c;  // next operand in flight
    x = o.mul(x, y);
    y = yn;
  }
  const bool one = tm_final_exp_is_one(o, x);
  if (gi < ngroups && c == 0) verdict[gi] = one ? 1 : 0;
}

// PublicKey.aggregate(...).toBytes(uncompressed) over cached keys through the verify
// path's own code: pk_sum of one slot (k_pk_agg's tree sum for >= BGV_PK_TREE_MIN keys,
// task_pk's serial sum below), then affine and the 96-byte ZCash encoding.
__global__ void k_pk_sum_out(const bgv_dslot* __restrict__ slot, const uint32_t* __restrict__ idx,
                             const g1_aff* __restrict__ cache, const g1_jac* __restrict__ pk_agg,
                             uint8_t* __restrict__ out96) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int32_t st = BGV_OK;
  const g1_jac acc = pk_sum(slot[0], idx, cache, nullptr, pk_agg, 0, &st);
  g1_aff a;
  const bool fin = jac_to_aff(&a, acc);
  uint8_t b[96];
  g1_serialize(b, a, !fin);
  for (int i = 0; i < 96; ++i) out96[i] = b[i];
}

// ---------------------------------------------------------------------------
// SURVEY 8(f) rows next to the verify path
// ---------------------------------------------------------------------------
// Deposit-time key validation (processDeposit.ts:62-69, PublicKey.fromBytes(pk, affine,
// validate=true)): ZCash decode, infinity -> BLST_PK_IS_INFINITY, [r]P != O ->
// BLST_POINT_NOT_IN_GROUP.  Valid keys are written as 96-B uncompressed records.
__device__ __noinline__ bool g1_in_subgroup(const g1_aff& a) {
  const uint32_t r[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                         0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  return jac_is_inf(jac_mul_u256(jac_from_aff(a), r));
}

__global__ void k_pk_validate(const uint8_t* __restrict__ keys48, uint32_t n, int32_t* __restrict__ status,
                              uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[48];
  for (int q = 0; q < 48; ++q) b[q] = keys48[48ull * i + q];
  g1_aff a;
  bool inf;
  int st = g1_decompress(&a, &inf, b);
  if (st == BGV_OK) {
    if (inf)
      st = BGV_PK_IS_INFINITY;
    else if (!g1_in_subgroup(a))
      st = BGV_POINT_NOT_IN_GROUP;
  }
  status[i] = st;
  uint8_t o[96];
  g1_serialize(o, a, st != BGV_OK);
  for (int q = 0; q < 96; ++q) out96[96ull * i + q] = o[q];
}

// Signature decode for aggregation (Signature.fromBytes(sig, undefined, true)): one
// signature per lane -> Jacobian point (infinity for the infinity encoding) + status.
__global__ void k_sig_decode(const uint8_t* __restrict__ sigs96, const uint32_t* __restrict__ lens, uint32_t n,
                             g2_jac* __restrict__ pts, int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t st = BGV_OK;
  g2_jac out = jac_infinity<fp2_t>();
  if (lens[i] != 96) {
    st = BGV_INVALID_SIZE;
  } else {
    uint8_t b[96];
    for (int q = 0; q < 96; ++q) b[q] = sigs96[96ull * i + q];
    g2_aff a;
    bool inf;
    st = g2_decompress(&a, &inf, b);
    if (st == BGV_OK && !inf) {
      const g2_jac j = jac_from_aff(a);
      if (g2_in_subgroup(j))
        out = j;
      else
        st = BGV_POINT_NOT_IN_GROUP;
    }
  }
  pts[i] = out;
  status[i] = st;
}

// One wavefront per aggregate: strided partial sums, then an LDS tree; compressed out.
__global__ void BGV_KATTR k_sig_sum(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count,
                                    const g2_jac* __restrict__ pts, uint8_t* __restrict__ out96) {
  extern __shared__ uint32_t lds[];
  g2_jac* ls = reinterpret_cast<g2_jac*>(lds);
  const uint32_t a = blockIdx.x, j = threadIdx.x, f = first[a], n = count[a];
  g2_jac acc = jac_infinity<fp2_t>();
  for (uint32_t k = j; k < n; k += BGV_WAVE) acc = jac_add(acc, pts[f + k]);
  for (uint32_t d = 1; d < BGV_WAVE; d <<= 1) {
    ls[j] = acc;
    __syncthreads();
    if ((j & (2 * d - 1)) == 0) acc = jac_add(acc, ls[j + d]);
    __syncthreads();
  }
  if (j == 0) {
    g2_aff r;
    const bool fin = jac_to_aff(&r, acc);
    uint8_t b[96];
    g2_compress(b, r, !fin);
    for (int q = 0; q < 96; ++q) out96[96ull * a + q] = b[q];
  }
}


__global__ void k_hash_msgs(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ offs,
                            const uint32_t* __restrict__ lens, uint32_t n, uint8_t* __restrict__ out192) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2_aff a;
  const bool fin = jac_to_aff(&a, hash_to_g2(msgs + offs[i], lens[i]));
  uint8_t b[192];
  g2_serialize(b, a, !fin);
  for (int k = 0; k < 192; ++k) out192[192ull * i + k] = b[k];
}

// 48-byte compressed pubkeys -> device cache entries (trusted, no subgroup check:
// state-transition/src/cache/pubkeyCache.ts:75 decompresses without validation)
__global__ void k_cache_put_compressed(const uint8_t* __restrict__ keys, uint32_t n, g1_aff* __restrict__ cache,
                                       int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[48];
  for (int k = 0; k < 48; ++k) b[k] = keys[48ull * i + k];
  g1_aff a;
  bool inf;
  int rc = g1_decompress(&a, &inf, b);
  if (rc == BGV_OK && inf) rc = BGV_PK_IS_INFINITY;
  if (rc == BGV_OK) cache[i] = a;
  status[i] = rc;
}

__global__ void k_cache_put_uncompressed(const uint8_t* __restrict__ keys, uint32_t n, g1_aff* __restrict__ cache,
                                         int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[96];
  for (int k = 0; k < 96; ++k) b[k] = keys[96ull * i + k];
  g1_aff a;
  bool inf;
  int rc = g1_deserialize(&a, &inf, b);
  if (rc == BGV_OK && inf) rc = BGV_PK_IS_INFINITY;
  if (rc == BGV_OK) cache[i] = a;
  status[i] = rc;
}


// ---------------------------------------------------------------------------
// Key generation and signing (bench / test data on the device; not on the
// verify path).  Secret keys are 32-byte big-endian scalars < r
// (SecretKey.fromBytes, state-transition/src/util/interop.ts:19-22).
// ---------------------------------------------------------------------------
__device__ static void sk_words(const uint8_t* be32, uint32_t k[8]) {
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = be32 + 28 - 4 * i;
    k[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

__global__ void k_keygen(const uint8_t* __restrict__ sks, uint32_t n, g1_aff* __restrict__ cache,
                         uint8_t* __restrict__ out48) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  sk_words(sks + 32ull * i, k);
  g1_aff a;
  const bool fin = jac_to_aff(&a, jac_mul_u256(jac_from_aff(g1_generator()), k));
  if (cache) cache[i] = a;
  if (out48) {
    uint8_t b[48];
    g1_compress(b, a, !fin);
    for (int q = 0; q < 48; ++q) out48[48ull * i + q] = b[q];
  }
}

__global__ void k_sign(const uint8_t* __restrict__ sks, const uint8_t* __restrict__ msgs, uint32_t n,
                       uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  sk_words(sks + 32ull * i, k);
  uint8_t m[32];
  for (int q = 0; q < 32; ++q) m[q] = msgs[32ull * i + q];
  g2_aff a;
  const bool fin = jac_to_aff(&a, jac_mul_u256(hash_to_g2(m, 32), k));
  uint8_t b[96];
  g2_compress(b, a, !fin);
  for (int q = 0; q < 96; ++q) out96[96ull * i + q] = b[q];
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Host-side launchers (declared in bgv_launch.h; called from bgv_api.cpp)
// ---------------------------------------------------------------------------
#include "bgv_launch.h"


static inline unsigned nblk(uint32_t n, unsigned t) { return (n + t - 1) / t; }

// Per-set kernels on one stream: k_prep (sig / hash / pk tasks side by side),
// then k_miller.  Kernel k is bracketed by events kev[2k], kev[2k+1] when profiling.
#define BGV_MARK(i) \
  if (s.kev) (void)hipEventRecord(s.kev[i], s.main)
hipError_t bgv_launch_prep(const bgv_dev_batch& b, const bgv_streams& s) {
  const uint32_t n = b.nslots;
  if (n == 0) return hipSuccess;
  BGV_MARK(0);
  // k_pk_agg only when some set is large enough; otherwise k_prep sums serially (null pk_agg)
  const bool tree = b.max_npk >= BGV_PK_TREE_MIN;
  if (tree)
    hipLaunchKernelGGL(k_pk_agg, dim3(n), dim3(64), 0, s.main, b.slots, n, b.pk_idx,
                       reinterpret_cast<const g1_aff*>(b.cache_opaque), b.pk_agg);
  hipLaunchKernelGGL(k_prep, dim3(nblk(n, 64), 3), dim3(64), 0, s.main, b.slots, n, b.rsig, b.sig_status, b.h,
                     b.pk_idx, reinterpret_cast<const g1_aff*>(b.cache_opaque), b.pk_bytes, b.rpk, b.pk_status,
                     tree ? b.pk_agg : nullptr);
  BGV_MARK(1);
  return hipGetLastError();
}

hipError_t bgv_launch_miller(const bgv_dev_batch& b, const bgv_streams& s) {
  const uint32_t n = b.nslots;
  if (n == 0) return hipSuccess;
  // the groups' signature sums, then set pairs and group pairs in one launch
  hipLaunchKernelGGL(k_gsum, dim3(nblk(b.ngroups, BGV_FINAL_TEAMS)), dim3(64), 0, s.main, b.groups, b.ngroups,
                     b.slots, b.rsig, b.sig_status, b.pk_status, b.gsum);
  BGV_MARK(2);
  hipLaunchKernelGGL(k_miller, dim3(nblk(n + b.ngroups, 64)), dim3(64), 0, s.main, b.slots, n, b.rpk, b.h,
                     b.sig_status, b.pk_status, b.f, b.ngroups, b.gsum, b.gpair);
  BGV_MARK(3);
  return hipGetLastError();
}

hipError_t bgv_launch_sets(const bgv_dev_batch& b, const bgv_streams& s) {
  hipError_t e = bgv_launch_prep(b, s);
  return e != hipSuccess ? e : bgv_launch_miller(b, s);
}

// Group closing over b.groups (contiguous slot ranges of <= 64 slots) after
// bgv_launch_miller (first pass, group pairs already made) or, for a retry round over the
// same per-slot results, with pairs = true: the parts' signature sums and pairs first.
hipError_t bgv_launch_groups(const bgv_dev_batch& b, const bgv_streams& s, bool pairs) {
  if (b.ngroups == 0) return hipSuccess;
  BGV_MARK(4);
  if (pairs) {
    hipLaunchKernelGGL(k_gsum, dim3(nblk(b.ngroups, BGV_FINAL_TEAMS)), dim3(64), 0, s.main, b.groups, b.ngroups,
                       b.slots, b.rsig, b.sig_status, b.pk_status, b.gsum);
    hipLaunchKernelGGL(k_gpair, dim3(nblk(b.ngroups, 64)), dim3(64), 0, s.main, b.ngroups, b.gsum, b.gpair);
  }
  hipLaunchKernelGGL(k_final, dim3(nblk(b.ngroups, BGV_FINAL_TEAMS)), dim3(64), 0, s.main, b.groups, b.ngroups,
                     b.f, b.gpair, b.verdict);
  BGV_MARK(5);
  return hipGetLastError();
}
#undef BGV_MARK

size_t bgv_slot_bytes() {
  return 2 * sizeof(g2_jac) + sizeof(g1_aff) + sizeof(fp12_t) + sizeof(g1_jac) + 2 * sizeof(int32_t);
}
size_t bgv_group_bytes() { return sizeof(g2_jac) + sizeof(fp12_t) + sizeof(int32_t); }
size_t bgv_cache_entry_bytes() { return sizeof(g1_aff); }

void bgv_carve(bgv_dev_batch* b, void* slot_mem, uint32_t cap_slots, void* group_mem, uint32_t cap_groups) {
  uint8_t* p = static_cast<uint8_t*>(slot_mem);
  b->rsig = reinterpret_cast<g2_jac*>(p);
  p += sizeof(g2_jac) * (size_t)cap_slots;
  b->h = reinterpret_cast<g2_jac*>(p);
  p += sizeof(g2_jac) * (size_t)cap_slots;
  b->rpk = reinterpret_cast<g1_aff*>(p);
  p += sizeof(g1_aff) * (size_t)cap_slots;
  b->f = reinterpret_cast<fp12_t*>(p);
  p += sizeof(fp12_t) * (size_t)cap_slots;
  b->pk_agg = reinterpret_cast<g1_jac*>(p);
  p += sizeof(g1_jac) * (size_t)cap_slots;
  b->sig_status = reinterpret_cast<int32_t*>(p);
  p += sizeof(int32_t) * (size_t)cap_slots;
  b->pk_status = reinterpret_cast<int32_t*>(p);
  uint8_t* q = static_cast<uint8_t*>(group_mem);
  b->gsum = reinterpret_cast<g2_jac*>(q);
  q += sizeof(g2_jac) * (size_t)cap_groups;
  b->gpair = reinterpret_cast<fp12_t*>(q);
  q += sizeof(fp12_t) * (size_t)cap_groups;
  b->verdict = reinterpret_cast<int32_t*>(q);
}

hipError_t bgv_launch_cache_put(const uint8_t* keys, uint32_t n, int fmt, bgv_cache_entry* cache, int32_t* status,
                                hipStream_t st) {
  if (n == 0) return hipSuccess;
  g1_aff* c = reinterpret_cast<g1_aff*>(cache);
  if (fmt == 48)
    hipLaunchKernelGGL(k_cache_put_compressed, dim3(nblk(n, 64)), dim3(64), 0, st, keys, n, c, status);
  else
    hipLaunchKernelGGL(k_cache_put_uncompressed, dim3(nblk(n, 64)), dim3(64), 0, st, keys, n, c, status);
  return hipGetLastError();
}

// slot: one device bgv_dslot {PK_CACHED, n_pk = n, pk_off = 0}; agg: one g1_jac of scratch
hipError_t bgv_launch_aggregate(const bgv_dslot* slot, const uint32_t* idx, uint32_t n, const bgv_cache_entry* cache,
                                void* agg, uint8_t* out96, hipStream_t st) {
  const g1_aff* c = reinterpret_cast<const g1_aff*>(cache);
  g1_jac* a = reinterpret_cast<g1_jac*>(agg);
  const bool tree = n >= BGV_PK_TREE_MIN;
  if (tree) hipLaunchKernelGGL(k_pk_agg, dim3(1), dim3(64), 0, st, slot, 1u, idx, c, a);
  hipLaunchKernelGGL(k_pk_sum_out, dim3(1), dim3(64), 0, st, slot, idx, c, tree ? a : nullptr, out96);
  return hipGetLastError();
}

hipError_t bgv_launch_hash(const uint8_t* msgs, const uint32_t* offs, const uint32_t* lens, uint32_t n,
                           uint8_t* out192, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hash_msgs, dim3(nblk(n, 64)), dim3(64), 0, st, msgs, offs, lens, n, out192);
  return hipGetLastError();
}

hipError_t bgv_launch_pk_validate(const uint8_t* keys48, uint32_t n, int32_t* status, uint8_t* out96,
                                  hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pk_validate, dim3(nblk(n, 64)), dim3(64), 0, st, keys48, n, status, out96);
  return hipGetLastError();
}

hipError_t bgv_launch_sig_aggregate(const uint8_t* sigs96, const uint32_t* lens, uint32_t n, const uint32_t* first,
                                    const uint32_t* count, uint32_t naggs, void* pts, int32_t* status,
                                    uint8_t* out96, hipStream_t st) {
  if (n) {
    hipLaunchKernelGGL(k_sig_decode, dim3(nblk(n, 64)), dim3(64), 0, st, sigs96, lens, n,
                       reinterpret_cast<g2_jac*>(pts), status);
  }
  if (naggs) {
    hipLaunchKernelGGL(k_sig_sum, dim3(naggs), dim3(64), BGV_WAVE * sizeof(g2_jac), st, first, count,
                       reinterpret_cast<const g2_jac*>(pts), out96);
  }
  return hipGetLastError();
}
size_t bgv_g2_point_bytes() { return sizeof(g2_jac); }
size_t bgv_g1_point_bytes() { return sizeof(g1_jac); }
hipError_t bgv_launch_keygen(const uint8_t* sks, uint32_t n, bgv_cache_entry* cache, uint8_t* out48, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_keygen, dim3(nblk(n, 64)), dim3(64), 0, st, sks, n, reinterpret_cast<g1_aff*>(cache), out48);
  return hipGetLastError();
}

hipError_t bgv_launch_sign(const uint8_t* sks, const uint8_t* msgs, uint32_t n, uint8_t* out96, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sign, dim3(nblk(n, 64)), dim3(64), 0, st, sks, msgs, n, out96);
  return hipGetLastError();
}
