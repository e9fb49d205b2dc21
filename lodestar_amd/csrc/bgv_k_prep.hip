// Per-set preparation kernels (gfx950) other than the bulk k_prep (bgv_k_prep_bulk.hip);
// see bgv_api.cpp for the launch order of a verify call and bgv_k_miller.hip /
// bgv_k_final.hip for the rest.
//
//   k_pk_agg16 / k_pk_agg  (only when a call holds a set with >= BGV_PK_TREE_MIN cached
//              keys) a team of 16 lanes per committee-sized set, a whole wavefront per set
//              above BGV_PK_TEAM_MAX keys, sums its keys with a ds_swizzle/ds_bpermute tree
//   k_prep_a / k_prep_team   the latency path for small calls (bgv_latency_max): the same
//              work over two launches with more lanes per set, so the longest chain per
//              lane roughly halves: (a) one SSWU map + isogeny per lane for u0 and u1, the
//              signature's decompression, the pubkey task; (team) the cofactor clearing of
//              q0 + q1 and r_i * sig_i on 16-lane teams, the subgroup check on one lane
//   k_prep     (bgv_k_prep_bulk.hip) sig, hash and pk tasks side by side for larger calls
#include "bgv_k_lat.h"
#include "bgv_team_dev.h"
#include "bgv_tcurve.h"
#include "bgv_tg1.h"
#include "bgv_tround_dev.h"

static __constant__ uint8_t kTcProg[TCP_TABLE_BYTES] = TCP_TABLE_INIT;
static __constant__ uint8_t kTg1Prog[TG1_TABLE_BYTES] = TG1_TABLE_INIT;

// Device engine of the team G2 schedules (bgv_tcurve.h): programs over the team's LDS slots
// with a block barrier per round; every team of the block runs the same sequence.
struct tc_dev_engine {
  const uint8_t* prog;
  fp_t* S;
  int c;
  bool bad;
  __device__ void run(int off) {
    int pos = off;
    const int nr = prog[pos++];
    for (int r = 0; r < nr; ++r) {
      const int T = prog[pos], M = prog[pos + 1];
      pos += 2;
      const int rb = tmp_rec_bytes(T, M);
      int out;
      const fp_t v = tmp_lane_any(S, prog + pos + c * rb, T, M, &out);
      S[out] = v;  // no slot is read and written in one round (tools/gen_tcurve.py)
      __syncthreads();
      pos += BGV_TEAM * rb;
    }
  }
  __device__ void copy(int dst, int src) {  // src may differ per team (a digit's table entry)
    if (c < 6 && dst != src) S[TCP_BANK(dst) + c] = S[TCP_BANK(src) + c];
    __syncthreads();
  }
  __device__ void neg_y(int b) {
    if (c == 2 || c == 3) S[TCP_BANK(b) + c] = fp_neg(S[TCP_BANK(b) + c]);
    __syncthreads();
  }
  __device__ void check_add() {
    if (c == 0) {
      const auto z2 = [&](int s) { return fp_is_zero(S[s]) && fp_is_zero(S[s + 1]); };
      bad = bad || z2(TC_CHK_A) || z2(TC_CHK_B);
    }
  }
};

#ifndef BGV_WPE_AGG
#define BGV_WPE_AGG 2
#endif

extern "C" {


// Pubkey aggregation of many-key sets as a wavefront tree (one wave per slot): lane l
// sums the set's cached keys l, l + 64, ... with mixed additions (coalesced gathers),
// then six butterfly levels of complete Jacobian additions with the partner lane's
// partial sum (lane ^ 32, 16, ..., 1) exchanged in registers.  Every lane ends with the
// total; the sum is the same group element as the serial one.  Waves of slots with fewer
// than BGV_PK_TREE_MIN cached keys exit at once (uniformly: every lane reads the same slot).
__device__ __forceinline__ void pk_aggw_body(const bgv_dslot* __restrict__ slots, uint32_t s,
                                             const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                             g1_jac* __restrict__ pk_agg) {
  const bgv_dslot& d = slots[s];
  if ((d.flags & BGV_SLOT_PAD) || !(d.flags & BGV_SLOT_PK_CACHED) || d.n_pk <= BGV_PK_TEAM_MAX) return;
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

__device__ __forceinline__ void pk_agg16_body(const bgv_dslot* __restrict__ slots, uint32_t nslots, uint32_t blk,
                                              const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                              g1_jac* __restrict__ pk_agg) {
  const uint32_t s = blk * (64 / 16) + threadIdx.x / 16;
  const uint32_t l = threadIdx.x % 16;
  const bgv_dslot* d = s < nslots ? &slots[s] : nullptr;
  const bool act = d && !(d->flags & BGV_SLOT_PAD) && (d->flags & BGV_SLOT_PK_CACHED) &&
                   d->n_pk >= BGV_PK_TREE_MIN && d->n_pk <= BGV_PK_TEAM_MAX;
  g1_jac acc = jac_infinity<fp_t>();
  if (act) {  // n_pk >= 16: every lane has a first key
    const uint32_t* idx = pk_idx + d->pk_off;
    const uint32_t n = d->n_pk;
    acc = jac_from_aff(cache[idx[l]]);
    uint32_t k = l + 16;
    g1_aff cur = cache[idx[k < n ? k : l]];
    for (; k < n; k += 16) {
      const uint32_t kn = k + 16 < n ? k + 16 : k;
      const g1_aff nxt = cache[idx[kn]];
      acc = jac_add_aff(acc, cur);
      cur = nxt;
    }
  }
  // every lane of the wave reaches the exchanges
  acc = jac_add(acc, point_xor<8>(acc));
  acc = jac_add(acc, point_xor<4>(acc));
  acc = jac_add(acc, point_xor<2>(acc));
  acc = jac_add(acc, point_xor<1>(acc));
  if (act && l == 0) pk_agg[s] = acc;
}

// One set's tree sum on a whole 64-lane block with the bulk path's summation order (so the
// same Jacobian representative, hence the same Miller value f): k_pk_agg16's 16-lane team for
// BGV_PK_TREE_MIN..BGV_PK_TEAM_MAX cached keys (lanes 16..63 repeat lanes 0..15), k_pk_agg's
// wave tree above.
__device__ __forceinline__ void pk_agg_one(const bgv_dslot* __restrict__ slots, uint32_t s,
                                           const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                           g1_jac* __restrict__ pk_agg) {
  const bgv_dslot& d = slots[s];
  if ((d.flags & BGV_SLOT_PAD) || !(d.flags & BGV_SLOT_PK_CACHED) || d.n_pk < BGV_PK_TREE_MIN) return;
  if (d.n_pk > BGV_PK_TEAM_MAX) {
    pk_aggw_body(slots, s, pk_idx, cache, pk_agg);
    return;
  }
  const uint32_t l = threadIdx.x % 16;
  const uint32_t* idx = pk_idx + d.pk_off;
  const uint32_t n = d.n_pk;
  g1_jac acc = jac_from_aff(cache[idx[l]]);
  for (uint32_t k = l + 16; k < n; k += 16) acc = jac_add_aff(acc, cache[idx[k]]);
  acc = jac_add(acc, point_xor<8>(acc));
  acc = jac_add(acc, point_xor<4>(acc));
  acc = jac_add(acc, point_xor<2>(acc));
  acc = jac_add(acc, point_xor<1>(acc));
  if (threadIdx.x == 0) pk_agg[s] = acc;
}

__global__ void __launch_bounds__(64) k_pk_agg(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                               const uint32_t* __restrict__ pk_idx,
                                               const g1_aff* __restrict__ cache, g1_jac* __restrict__ pk_agg) {
  if (blockIdx.x < nslots) pk_aggw_body(slots, blockIdx.x, pk_idx, cache, pk_agg);
}

// The latency path's first launch for calls above BGV_PREP_WIDE_MAX sets (the smallest calls
// run k_prep_a_wave, bgv_k_prep_wave.hip): planes 0..2 the maps of u0 / u1 and the signature's
// decoding, one lane per set, plane 3 the pubkey task.
__global__ void BGV_KATTR_PREP k_prep_a(const bgv_dslot* __restrict__ slots, uint32_t nslots, g2_jac* __restrict__ h,
                                        fp12_t* __restrict__ f, int32_t* __restrict__ sig_status,
                                        const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                        const uint8_t* __restrict__ pk_bytes, g1_jac* __restrict__ rpk,
                                        int32_t* __restrict__ pk_status, g1_jac* __restrict__ pk_agg) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  if (blockIdx.y == 0)
    task_map_t<bgv_pow_lane>(s, 0, slots, h + s, true);
  else if (blockIdx.y == 1)
    task_map_t<bgv_pow_lane>(s, 1, slots, split_q1(f, s), true);
  else if (blockIdx.y == 2)
    task_sig_decode_t<bgv_pow_lane>(s, slots, split_sig(f, s), sig_status, true);
  else
    task_pk(s, slots, pk_idx, cache, pk_bytes, rpk, pk_status, pk_agg);
}

// The latency path's second launch on teams (bgv_tcurve.h): blockIdx.y = 0 the cofactor
// clearing of q0 + q1 (one team per set), 1 r_i * sig_i (one team per set), 2 the
// signature's subgroup check (one lane per set).  A team whose cofactor clearing met an
// exceptional addition recomputes it on one lane with the complete formulas.
__global__ void __launch_bounds__(64) k_prep_team(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                                  g2_jac* __restrict__ h, fp12_t* __restrict__ f,
                                                  g2_jac* __restrict__ rsig, int32_t* __restrict__ sig_status) {
  if (blockIdx.y == 2) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslots || (slots[s].flags & BGV_SLOT_PAD) || sig_status[s] != BGV_ST_OK) return;
    if (!g2_in_subgroup(jac_from_aff(*split_sig(f, s)))) sig_status[s] = BGV_POINT_NOT_IN_GROUP;
    return;
  }
  __shared__ uint8_t prog[TCP_TABLE_BYTES];
  __shared__ fp_t Sall[BGV_FINAL_TEAMS][TCP_NSLOT];
  __shared__ int flags[BGV_FINAL_TEAMS];
  for (int i = threadIdx.x; i < TCP_TABLE_BYTES; i += 64) prog[i] = kTcProg[i];
  const int team = threadIdx.x / BGV_TEAM, c = threadIdx.x % BGV_TEAM;
  const uint32_t u = blockIdx.x * BGV_FINAL_TEAMS + team;
  const uint32_t uu = u < nslots ? u : nslots - 1;
  const bgv_dslot& d = slots[uu];
  const bool real = u < nslots && !(d.flags & BGV_SLOT_PAD);
  fp_t* S = Sall[team];
  if (c == 6) {
    S[TCP_S_ONE] = fp_one();
  } else if (c >= 7 && c < 11) {
    const fp2_t cx = BGV_PSI_CX, cy = BGV_PSI_CY;
    const fp2_t& v = c < 9 ? cx : cy;
    S[c < 9 ? TCP_S_PSI_CX + (c - 7) : TCP_S_PSI_CY + (c - 9)] = (c & 1) ? v.c0 : v.c1;
  } else if (c == 11) {
    S[TCP_S_PSI2_CX] = fp_t{BGV_PSI2_CX};
  } else if (c == 12) {
    S[TCP_S_PSI2_CY] = fp_t{BGV_PSI2_CY};
  }
  for (int i = c; i < TC_ISO_NCONST; i += BGV_TEAM) S[TCP_S_ISO + i] = tc_iso_const(i);
  tc_dev_engine e{prog, S, c, false};
  if (blockIdx.y == 0) {
    if (c < 6) {
      S[TCP_BANK(1) + c] = reinterpret_cast<const fp_t*>(h + uu)[c];
      S[TCP_BANK(2) + c] = reinterpret_cast<const fp_t*>(split_q1(f, uu))[c];
    }
    __syncthreads();
    tc_clear_cofactor(e);
    if (c == 0) flags[team] = e.bad ? 1 : 0;
    __syncthreads();
    if (real) {
      if (!flags[team]) {
        if (c < 6) reinterpret_cast<fp_t*>(h + uu)[c] = S[TCP_BANK(3) + c];
      } else if (c == 0) {
        h[uu] = g2_clear_cofactor(jac_add(iso_map_g2_jac(h[uu]), iso_map_g2_jac(*split_q1(f, uu))));
      }
    }
  } else {
    const bool ok = sig_status[uu] == BGV_ST_OK;  // the decode left it OK (the subgroup lanes may flip it)
    if (c < 4)
      S[TCP_BANK(1) + c] = reinterpret_cast<const fp_t*>(split_sig(f, uu))[c];
    else if (c < 6)
      S[TCP_BANK(1) + c] = c == 4 ? fp_one() : fp_zero();
    __syncthreads();
    tc_mul_glv(e, d.scalar);
    if (real && ok && c < 6) reinterpret_cast<fp_t*>(rsig + uu)[c] = S[TCP_BANK(4) + c];
  }
}

// The point-program engine of bgv_tcurve.h's schedules on a whole block (bgv_tround_dev.h:
// four-part round instructions): bank moves by the q = 0 lanes, one block per set.
struct tc_wide_engine : tr_wide_engine {
  __device__ void copy(int dst, int src) {
    if (q == 0 && c < 6 && dst != src) S[TCP_BANK(dst) + c] = S[TCP_BANK(src) + c];
    __syncthreads();
  }
  __device__ void neg_y(int b) {
    if (q == 0 && (c == 2 || c == 3)) S[TCP_BANK(b) + c] = fp_neg(S[TCP_BANK(b) + c]);
    __syncthreads();
  }
  __device__ void check_add() {
    if (q == 0 && c == 0) {
      const auto z2 = [&](int s) { return fp_is_zero(S[s]) && fp_is_zero(S[s + 1]); };
      bad = bad || z2(TC_CHK_A) || z2(TC_CHK_B);
    }
  }
};

// The G1 schedule (bgv_tg1.h) on the same four-part engine: three-slot banks.
struct tg1_wide_engine : tr_wide_engine {
  __device__ void copy(int dst, int src) {
    if (q == 0 && c < 3 && dst != src) S[TG1_BANK(dst) + c] = S[TG1_BANK(src) + c];
    __syncthreads();
  }
};

// k_prep_team for the smallest calls, one set per 64-lane block and task (blockIdx.y): 0 the
// cofactor clearing of q0 + q1, 1 r_i * sig_i, 2 the signature's subgroup check psi(P) ==
// [x]P with [|x|]P from the same point programs (a team-level exceptional addition falls
// back to the one-lane g2_in_subgroup).  Same schedules and formulas as k_prep_team.
__global__ void __launch_bounds__(64) k_prep_wide(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                                  g2_jac* __restrict__ h, fp12_t* __restrict__ f,
                                                  g2_jac* __restrict__ rsig, int32_t* __restrict__ sig_status,
                                                  const uint32_t* __restrict__ pk_idx,
                                                  const g1_aff* __restrict__ cache, const uint8_t* __restrict__ pk_bytes,
                                                  g1_jac* __restrict__ rpk, int32_t* __restrict__ pk_status,
                                                  g1_jac* __restrict__ pk_agg) {
  static_assert(TG1_TABLE_BYTES <= TCP_TABLE_BYTES && TG1_NSLOT <= TCP_NSLOT, "plane 3 reuses the G2 buffers");
  __shared__ uint8_t prog[TCP_TABLE_BYTES];
  __shared__ fp_t S[TCP_NSLOT];
  __shared__ fp_t RP[64];
  __shared__ int flag;
  if (blockIdx.y == 3) {  // the pubkey task, one set per block
    // a set of >= BGV_PK_TREE_MIN cached keys first sums them on the whole wave (k_pk_agg's
    // tree); lane 0 then takes the set's sum and status, and r * sum runs on the G1 point
    // programs (bgv_tg1.h) as rounds, concurrently with the other planes' G2 programs
    const uint32_t s = blockIdx.x;
    if (pk_agg) pk_agg_one(slots, s, pk_idx, cache, pk_agg);
    if (threadIdx.x == 0) {
      g1_jac acc;
      const bool go = task_pk_sum(s, slots, pk_idx, cache, pk_bytes, pk_status, pk_agg, &acc);
      flag = go ? 1 : 0;
      if (go) {
        S[TG1_BANK(1)] = acc.x;
        S[TG1_BANK(1) + 1] = acc.y;
        S[TG1_BANK(1) + 2] = acc.z;
      }
      S[TG1_S_ONE] = fp_one();
      S[TG1_S_BETA] = fp_t{BGV_BETA_MX2};
    }
    for (int i = threadIdx.x; i < TG1_TABLE_BYTES; i += 64) prog[i] = kTg1Prog[i];
    __syncthreads();
    if (!flag) return;  // uniform over the block
    const int lane = threadIdx.x;
    tg1_wide_engine e{{prog, S, RP, tr_wide_lane_c(lane), tr_wide_lane_q(lane), false}};
    tg1_mul_glv(e, slots[s].scalar);
    if (lane < 3) reinterpret_cast<fp_t*>(rpk + s)[lane] = S[TG1_BANK(4) + lane];
    if (lane == 0) pk_status[s] = BGV_ST_OK;
    return;
  }
  const uint32_t uu = blockIdx.x;  // grid = exactly nslots blocks per task
  const int lane = threadIdx.x, c = lane % BGV_TEAM, q = lane / BGV_TEAM;
  const bgv_dslot& d = slots[uu];
  const bool real = !(d.flags & BGV_SLOT_PAD);
  // the subgroup check only for signatures that decoded to a finite point (uniform per block)
  if (blockIdx.y == 2 && (!real || sig_status[uu] != BGV_ST_OK)) return;
  for (int i = lane; i < TCP_TABLE_BYTES; i += 64) prog[i] = kTcProg[i];
  if (q == 0) {
    if (c == 6) {
      S[TCP_S_ONE] = fp_one();
    } else if (c >= 7 && c < 11) {
      const fp2_t cx = BGV_PSI_CX, cy = BGV_PSI_CY;
      const fp2_t& v = c < 9 ? cx : cy;
      S[c < 9 ? TCP_S_PSI_CX + (c - 7) : TCP_S_PSI_CY + (c - 9)] = (c & 1) ? v.c0 : v.c1;
    } else if (c == 11) {
      S[TCP_S_PSI2_CX] = fp_t{BGV_PSI2_CX};
    } else if (c == 12) {
      S[TCP_S_PSI2_CY] = fp_t{BGV_PSI2_CY};
    }
  }
  for (int i = lane; i < TC_ISO_NCONST; i += 64) S[TCP_S_ISO + i] = tc_iso_const(i);
  tc_wide_engine e{{prog, S, RP, tr_wide_lane_c(lane), tr_wide_lane_q(lane), false}};
  if (blockIdx.y == 0) {
    if (q == 0 && c < 6) {
      S[TCP_BANK(1) + c] = reinterpret_cast<const fp_t*>(h + uu)[c];
      S[TCP_BANK(2) + c] = reinterpret_cast<const fp_t*>(split_q1(f, uu))[c];
    }
    __syncthreads();
    tc_clear_cofactor(e);
    if (lane == 0) flag = e.bad ? 1 : 0;
    __syncthreads();
    if (real) {
      if (!flag) {
        if (q == 0 && c < 6) reinterpret_cast<fp_t*>(h + uu)[c] = S[TCP_BANK(3) + c];
      } else if (lane == 0) {
        h[uu] = g2_clear_cofactor(jac_add(iso_map_g2_jac(h[uu]), iso_map_g2_jac(*split_q1(f, uu))));
      }
    }
  } else if (blockIdx.y == 1) {
    const bool ok = sig_status[uu] == BGV_ST_OK;  // read before the subgroup blocks may flip it
    if (q == 0) {
      if (c < 4)
        S[TCP_BANK(1) + c] = reinterpret_cast<const fp_t*>(split_sig(f, uu))[c];
      else if (c < 6)
        S[TCP_BANK(1) + c] = c == 4 ? fp_one() : fp_zero();
    }
    __syncthreads();
    tc_mul_glv(e, d.scalar);
    if (real && ok && q == 0 && c < 6) reinterpret_cast<fp_t*>(rsig + uu)[c] = S[TCP_BANK(4) + c];
  } else {
    // [|x|]P: base in bank 0, the accumulator (= P) in bank 4
    if (q == 0 && c < 6) {
      const fp_t v = c < 4 ? reinterpret_cast<const fp_t*>(split_sig(f, uu))[c] : (c == 4 ? fp_one() : fp_zero());
      S[TCP_BANK(0) + c] = v;
      S[TCP_BANK(4) + c] = v;
    }
    __syncthreads();
    const int a = tc_to_jac(e, tc_mul_x_abs(e));
    if (lane == 0) {
      const g2_jac p = jac_from_aff(*split_sig(f, uu));
      bool in;
      if (e.bad) {
        in = g2_in_subgroup(p);
      } else {
        const fp_t* B = S + TCP_BANK(a);
        const g2_jac xp = {{B[0], B[1]}, {B[2], B[3]}, {B[4], B[5]}};
        in = jac_eq(g2_psi(p), jac_neg(xp));  // psi(P) == [x]P = -[|x|]P
      }
      if (!in) sig_status[uu] = BGV_POINT_NOT_IN_GROUP;
    }
  }
}

// Committee-sized sets (BGV_PK_TREE_MIN..BGV_PK_TEAM_MAX cached keys, e.g. 128-key
// attestation aggregates) on a team of 16 lanes, four sets per wave: lane l sums keys
// l, l + 16, ... with mixed additions, then four ds_swizzle butterfly levels (xor 8..1, inside
// the team).  A whole wave per 128-key set spent ~4x the lane work on the tree levels.
// The lane's first key starts the sum (no addition to infinity), and each key is gathered
// one addition ahead of its use.  A gather-latency-bound kernel: BGV_WPE_AGG waves per SIMD.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE_AGG, BGV_WPE_AGG)))
k_pk_agg16(const bgv_dslot* __restrict__ slots, uint32_t nslots, const uint32_t* __restrict__ pk_idx,
           const g1_aff* __restrict__ cache, g1_jac* __restrict__ pk_agg) {
  pk_agg16_body(slots, nslots, blockIdx.x, pk_idx, cache, pk_agg);
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

}  // extern "C"

hipError_t bgv_launch_prep(const bgv_dev_batch& b, const bgv_streams& s) {
  const uint32_t n = b.nslots;
  if (n == 0) return hipSuccess;
  BGV_MARK(0);
  // k_pk_agg only when some set is large enough; otherwise k_prep sums serially (null pk_agg)
  const bool tree = b.max_npk >= BGV_PK_TREE_MIN;
  const bool wide = bgv_use_latency(b, n + b.ngroups) && n <= BGV_PREP_WIDE_MAX;
  if (wide) {
    const g1_aff* cache = reinterpret_cast<const g1_aff*>(b.cache_opaque);
    const hipError_t e = bgv_launch_prep_wave(b, s.main);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_prep_wide, dim3(n, 4), dim3(64), 0, s.main, b.slots, n, b.h, b.f, b.rsig, b.sig_status,
                       b.pk_idx, cache, b.pk_bytes, b.rpk, b.pk_status, tree ? b.pk_agg : nullptr);
    BGV_MARK(1);
    return hipGetLastError();
  }
  if (tree)
    hipLaunchKernelGGL(k_pk_agg16, dim3(nblk(n, 4)), dim3(64), 0, s.main, b.slots, n, b.pk_idx,
                       reinterpret_cast<const g1_aff*>(b.cache_opaque), b.pk_agg);
  if (b.max_npk > BGV_PK_TEAM_MAX)
    hipLaunchKernelGGL(k_pk_agg, dim3(n), dim3(64), 0, s.main, b.slots, n, b.pk_idx,
                       reinterpret_cast<const g1_aff*>(b.cache_opaque), b.pk_agg);
  if (bgv_use_latency(b, n + b.ngroups)) {
    hipLaunchKernelGGL(k_prep_a, dim3(nblk(n, 64), 4), dim3(64), 0, s.main, b.slots, n, b.h, b.f, b.sig_status,
                       b.pk_idx, reinterpret_cast<const g1_aff*>(b.cache_opaque), b.pk_bytes, b.rpk, b.pk_status,
                       tree ? b.pk_agg : nullptr);
    hipLaunchKernelGGL(k_prep_team, dim3(nblk(n, BGV_FINAL_TEAMS), 3), dim3(64), 0, s.main, b.slots, n, b.h, b.f,
                       b.rsig, b.sig_status);
  } else {
    const hipError_t e = bgv_launch_prep_bulk(b, s, tree);
    if (e != hipSuccess) return e;
  }
  BGV_MARK(1);
  return hipGetLastError();
}

// slot: one device bgv_dslot {PK_CACHED, n_pk = n, pk_off = 0}; agg: one g1_jac of scratch
hipError_t bgv_launch_aggregate(const bgv_dslot* slot, const uint32_t* idx, uint32_t n, const bgv_cache_entry* cache,
                                void* agg, uint8_t* out96, hipStream_t st) {
  const g1_aff* c = reinterpret_cast<const g1_aff*>(cache);
  g1_jac* a = reinterpret_cast<g1_jac*>(agg);
  const bool tree = n >= BGV_PK_TREE_MIN;
  if (tree && n <= BGV_PK_TEAM_MAX) hipLaunchKernelGGL(k_pk_agg16, dim3(1), dim3(64), 0, st, slot, 1u, idx, c, a);
  if (tree && n > BGV_PK_TEAM_MAX) hipLaunchKernelGGL(k_pk_agg, dim3(1), dim3(64), 0, st, slot, 1u, idx, c, a);
  hipLaunchKernelGGL(k_pk_sum_out, dim3(1), dim3(64), 0, st, slot, idx, c, tree ? a : nullptr, out96);
  return hipGetLastError();
}
