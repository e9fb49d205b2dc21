// Batch BLS12-381 signature-set verification kernels for CDNA4 (gfx950).
//
// One signature set per lane.  A verify call runs these kernels in order (see
// bgv_api.cpp):
//
//   k_prep     three independent tasks side by side (blockIdx.y):
//              sig  decompress + subgroup-check the 96-byte signature -> affine sig_i
//              hash hash_to_G2(signing root) -> affine H(m_i)
//              pk   gather + aggregate pubkeys from the device cache; r_i * pk_i and
//                   r_i * (-G1), both made affine with one shared inversion
//   k_miller   f_i = MillerLoop(r_i pk_i, H(m_i)) * MillerLoop(-r_i G1, sig_i), one
//              shared Fp12 accumulator (2-pair loop)
//   k_final    per device group (a team of 16 lanes): prod f_i over the group's
//              slots, then the final-exponentiation check -> == 1
//
// This is the randomized batch equation of blst's verifyMultipleAggregateSignatures
// (called from packages/beacon-node/src/chain/bls/maybeBatch.ts:18-25):
//   prod_i e(r_i pk_i, H(m_i)) * e(-G1, sum_i r_i sig_i) == 1,
// with e(-G1, sum r_i sig_i) = prod_i e(-r_i G1, sig_i) moved into the per-set
// kernel, so a group closes with a product and one final exponentiation only.
// A one-set group is the core verify of maybeBatch.ts:34-38 raised to the
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

extern "C" {

__device__ __noinline__ void task_sig(uint32_t s, const bgv_dslot* __restrict__ slots, g2_aff* __restrict__ sig,
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
      if (inf)
        st = BGV_ST_INFINITY;  // skipped in the accumulator, as blst does
      else if (!g2_in_subgroup(jac_from_aff(a)))
        st = BGV_POINT_NOT_IN_GROUP;
      else
        sig[s] = a;
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

__device__ __noinline__ void task_pk(uint32_t s, const bgv_dslot* __restrict__ slots,
                                     const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                     const uint8_t* __restrict__ pk_bytes, g1_aff* __restrict__ rpk,
                                     g1_aff* __restrict__ rg, int32_t* __restrict__ pk_status,
                                     const g1_aff* __restrict__ gtab, const g1_jac* __restrict__ pk_agg) {
  const bgv_dslot& d = slots[s];
  int32_t st = BGV_ST_OK;
  if (d.flags & BGV_SLOT_PAD) {
    pk_status[s] = BGV_ST_INFINITY;
    return;
  }
  g1_jac acc = jac_infinity<fp_t>();
  const bool cached = (d.flags & BGV_SLOT_PK_CACHED) != 0;
  const bool tree = pk_agg != nullptr && cached && d.n_pk >= BGV_PK_TREE_MIN;  // summed by k_pk_agg
  if (tree) acc = pk_agg[s];
  for (uint32_t k = 0; k < (tree ? 0u : d.n_pk); ++k) {
    g1_aff a;
    if (cached) {
      a = cache[pk_idx[d.pk_off + k]];
    } else {
      uint8_t b[96];
      const uint8_t* src = pk_bytes + 96ull * (d.pk_off + k);
      for (int i = 0; i < 96; ++i) b[i] = src[i];
      bool inf;
      const int rc = g1_deserialize(&a, &inf, b);
      if (rc == BGV_OK && !inf && !g1_aff_on_curve(a)) st = BGV_POINT_NOT_ON_CURVE;
      else if (rc != BGV_OK) st = rc;
      if (st != BGV_OK) break;
      if (inf) continue;
    }
    acc = jac_add_aff(acc, a);
  }
  if (st == BGV_OK) {
    const g1_jac a = jac_mul_u64(acc, d.scalar);
    if (jac_is_inf(a)) {
      st = BGV_ST_INFINITY;
    } else {
      // r_i * (-G1) for the signature's pair from the fixed-base table; never infinity
      // (0 < r_i < group order)
      const g1_jac g = g1_neg_gen_mul(gtab, d.scalar);
      g1_aff pa, ga;
      jac2_to_aff(&pa, &ga, a, g);
      rpk[s] = pa;
      rg[s] = ga;
    }
  }
  pk_status[s] = st;
}

// Pubkey aggregation of many-key sets as a wavefront tree (one wave per slot): lane l
// sums the set's cached keys l, l + 64, ... with mixed additions (coalesced gathers),
// then six levels of complete Jacobian additions through LDS.  The sum is the same group
// element as the serial one, so r * pk and its affine bytes are unchanged.  Waves of
// slots with fewer than BGV_PK_TREE_MIN cached keys exit at once (uniformly: every lane
// reads the same slot), so no barrier is left waiting.
__global__ void __launch_bounds__(64) k_pk_agg(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                               const uint32_t* __restrict__ pk_idx,
                                               const g1_aff* __restrict__ cache, g1_jac* __restrict__ pk_agg) {
  const uint32_t s = blockIdx.x;
  if (s >= nslots) return;
  const bgv_dslot& d = slots[s];
  if ((d.flags & BGV_SLOT_PAD) || !(d.flags & BGV_SLOT_PK_CACHED) || d.n_pk < BGV_PK_TREE_MIN) return;
  __shared__ g1_jac t[64];
  const uint32_t l = threadIdx.x;
  g1_jac acc = jac_infinity<fp_t>();
  for (uint32_t k = l; k < d.n_pk; k += 64) acc = jac_add_aff(acc, cache[pk_idx[d.pk_off + k]]);
  t[l] = acc;
  __syncthreads();
  for (uint32_t off = 32; off > 0; off >>= 1) {
    if (l < off) t[l] = jac_add(t[l], t[l + off]);
    __syncthreads();
  }
  if (l == 0) pk_agg[s] = t[0];
}

// The three independent per-set tasks in one launch (blockIdx.y = task), so one
// batch keeps 3x the wavefronts in flight on a single stream.
__global__ void BGV_KATTR_PREP k_prep(const bgv_dslot* __restrict__ slots, uint32_t nslots, g2_aff* __restrict__ sig,
                                 int32_t* __restrict__ sig_status, g2_jac* __restrict__ h,
                                 const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                 const uint8_t* __restrict__ pk_bytes, g1_aff* __restrict__ rpk,
                                 g1_aff* __restrict__ rg, int32_t* __restrict__ pk_status,
                                 const g1_aff* __restrict__ gtab, const g1_jac* __restrict__ pk_agg) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  // hash first: the longest task starts earliest
  if (blockIdx.y == 0)
    task_hash(s, slots, h);
  else if (blockIdx.y == 1)
    task_sig(s, slots, sig, sig_status);
  else
    task_pk(s, slots, pk_idx, cache, pk_bytes, rpk, rg, pk_status, gtab, pk_agg);
}

// k_miller lives in bgv_miller_kernel.h; -DBGV_MILLER_SPLIT compiles it in its own
// translation unit (bgv_kernels_miller.hip) with the Fp products inlined.
#ifdef BGV_MILLER_SPLIT
__global__ void BGV_KATTR k_miller(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                   const g1_aff* __restrict__ rpk, const g2_jac* __restrict__ h,
                                   const g1_aff* __restrict__ rg, const g2_aff* __restrict__ sig,
                                   const int32_t* __restrict__ sig_status, const int32_t* __restrict__ pk_status,
                                   fp12_t* __restrict__ f);
#else
#include "bgv_miller_kernel.h"
#endif

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
// One team per device group: the product of the group's per-slot f_i (coefficient-
// parallel team products, operands straight from the per-slot array), then the
// final-exponentiation check.  The teams of a wave loop to the wave's longest group,
// the shorter ones multiplying by 1, so every lane reaches every barrier.
__global__ void BGV_KATTR k_final(const bgv_dgroup* __restrict__ groups, uint32_t ngroups,
                                  const fp12_t* __restrict__ f, int32_t* __restrict__ verdict) {
  __shared__ fp_t lds[BGV_FINAL_TEAMS][2 * BGV_TEAM_COMPS];
  __shared__ uint32_t lens[BGV_FINAL_TEAMS];
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const int cc = c < BGV_TEAM_COMPS ? c : c - 4;
  const uint32_t gi = blockIdx.x * BGV_FINAL_TEAMS + team;
  // teams past the end duplicate the last group
  const bgv_dgroup g = groups[gi < ngroups ? gi : ngroups - 1];
  if (c == 0) lens[team] = g.n_slots;
  __syncthreads();
  uint32_t nmax = 0;
  BGV_UNROLL for (int t = 0; t < BGV_FINAL_TEAMS; ++t) nmax = lens[t] > nmax ? lens[t] : nmax;
  const int fi = tm_fp_index(cc);
  const fp_t one_c = cc == 0 ? fp_one() : fp_zero();  // component cc of 1
  const fp_t* fs = reinterpret_cast<const fp_t*>(f + g.first_slot);
  constexpr int kFp12 = (int)(sizeof(fp12_t) / sizeof(fp_t));
  tm_dev_ops o{lds[team], lds[team] + BGV_TEAM_COMPS, c, cc};
  fp_t x = g.n_slots ? fs[fi] : one_c;
  fp_t y = 1 < g.n_slots ? fs[kFp12 + fi] : one_c;
  BGV_NO_UNROLL for (uint32_t k = 1; k < nmax; ++k) {
    const fp_t yn = k + 1 < g.n_slots ? fs[kFp12 * (k + 1) + fi] : one_c;  // next operand in flight
    x = o.mul(x, y);
    y = yn;
  }
  const bool one = tm_final_exp_is_one(o, x);
  if (gi < ngroups && c == 0) verdict[gi] = one ? 1 : 0;
}

__global__ void k_aggregate_cached(const uint32_t* __restrict__ idx, uint32_t n, const g1_aff* __restrict__ cache,
                                   uint8_t* __restrict__ out96) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  g1_jac acc = jac_infinity<fp_t>();
  for (uint32_t k = 0; k < n; ++k) acc = jac_add_aff(acc, cache[idx[k]]);
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

__global__ void k_gtab_build(g1_aff* __restrict__ tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < BGV_GTAB_ENTRIES) tab[i] = g1_gtab_entry(i);
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
  if (rc == BGV_OK && !g1_aff_on_curve(a)) rc = BGV_POINT_NOT_ON_CURVE;
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
  hipLaunchKernelGGL(k_prep, dim3(nblk(n, 64), 3), dim3(64), 0, s.main, b.slots, n, b.sig, b.sig_status, b.h,
                     b.pk_idx, reinterpret_cast<const g1_aff*>(b.cache_opaque), b.pk_bytes, b.rpk, b.rg,
                     b.pk_status, reinterpret_cast<const g1_aff*>(b.gtab), tree ? b.pk_agg : nullptr);
  BGV_MARK(1);
  return hipGetLastError();
}

hipError_t bgv_launch_miller(const bgv_dev_batch& b, const bgv_streams& s) {
  const uint32_t n = b.nslots;
  if (n == 0) return hipSuccess;
  BGV_MARK(2);
  hipLaunchKernelGGL(k_miller, dim3(nblk(n, 64)), dim3(64), 0, s.main, b.slots, n, b.rpk, b.h, b.rg, b.sig,
                     b.sig_status, b.pk_status, b.f);
  BGV_MARK(3);
  return hipGetLastError();
}

hipError_t bgv_launch_sets(const bgv_dev_batch& b, const bgv_streams& s) {
  hipError_t e = bgv_launch_prep(b, s);
  return e != hipSuccess ? e : bgv_launch_miller(b, s);
}

// Per-group kernels over b.groups (contiguous slot ranges of <= 64 slots): used for
// the first pass and, over the same per-slot results, for the per-job retry pass.
hipError_t bgv_launch_groups(const bgv_dev_batch& b, const bgv_streams& s) {
  if (b.ngroups == 0) return hipSuccess;
  BGV_MARK(4);
  hipLaunchKernelGGL(k_final, dim3(nblk(b.ngroups, BGV_FINAL_TEAMS)), dim3(64), 0, s.main, b.groups, b.ngroups, b.f,
                     b.verdict);
  BGV_MARK(5);
  return hipGetLastError();
}
#undef BGV_MARK

size_t bgv_slot_bytes() {
  return sizeof(g2_aff) + sizeof(g2_jac) + 2 * sizeof(g1_aff) + sizeof(fp12_t) + sizeof(g1_jac) +
         2 * sizeof(int32_t);
}
size_t bgv_group_bytes() { return sizeof(int32_t); }
size_t bgv_cache_entry_bytes() { return sizeof(g1_aff); }

void bgv_carve(bgv_dev_batch* b, void* slot_mem, uint32_t cap_slots, void* group_mem, uint32_t cap_groups) {
  uint8_t* p = static_cast<uint8_t*>(slot_mem);
  b->sig = reinterpret_cast<g2_aff*>(p);
  p += sizeof(g2_aff) * (size_t)cap_slots;
  b->h = reinterpret_cast<g2_jac*>(p);
  p += sizeof(g2_jac) * (size_t)cap_slots;
  b->rpk = reinterpret_cast<g1_aff*>(p);
  p += sizeof(g1_aff) * (size_t)cap_slots;
  b->rg = reinterpret_cast<g1_aff*>(p);
  p += sizeof(g1_aff) * (size_t)cap_slots;
  b->f = reinterpret_cast<fp12_t*>(p);
  p += sizeof(fp12_t) * (size_t)cap_slots;
  b->pk_agg = reinterpret_cast<g1_jac*>(p);
  p += sizeof(g1_jac) * (size_t)cap_slots;
  b->sig_status = reinterpret_cast<int32_t*>(p);
  p += sizeof(int32_t) * (size_t)cap_slots;
  b->pk_status = reinterpret_cast<int32_t*>(p);
  (void)cap_groups;
  b->verdict = static_cast<int32_t*>(group_mem);
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

hipError_t bgv_launch_aggregate(const uint32_t* idx, uint32_t n, const bgv_cache_entry* cache, uint8_t* out96,
                                hipStream_t st) {
  hipLaunchKernelGGL(k_aggregate_cached, dim3(1), dim3(64), 0, st, idx, n, reinterpret_cast<const g1_aff*>(cache),
                     out96);
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
size_t bgv_gtab_bytes() { return sizeof(g1_aff) * BGV_GTAB_ENTRIES; }
hipError_t bgv_launch_gtab(void* tab, hipStream_t st) {
  hipLaunchKernelGGL(k_gtab_build, dim3(BGV_GTAB_ENTRIES / 64), dim3(64), 0, st, reinterpret_cast<g1_aff*>(tab));
  return hipGetLastError();
}

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
