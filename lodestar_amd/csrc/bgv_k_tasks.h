// Per-set tasks of the preparation kernels, shared by the bulk k_prep unit
// (bgv_k_prep_bulk.hip) and the latency-path / parity-hook unit (bgv_k_prep.hip).  Each unit
// compiles its own copy (no device linking), so each gets its own register budget.
//   task_sig   decompress + subgroup-check the 96-byte signature, then r_i * sig_i
//   task_hash  hash_to_G2(signing root) -> H(m_i), Jacobian
//   task_pk    gather + aggregate pubkeys from the device cache; r_i * pk_i (Jacobian)
#pragma once
#include "bgv_device.h"

// r_i * sig_i of a set whose signature decodes and lies in G2 (else only a status).
static __device__ __noinline__ void task_sig(uint32_t s, const bgv_dslot* __restrict__ slots, g2_jac* __restrict__ rsig,
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
          rsig[s] = jac_mul_glv(j, d.scalar);  // never infinity: 0 < r < group order
      }
    }
  }
  sig_status[s] = st;
}

static __device__ __noinline__ void task_hash(uint32_t s, const bgv_dslot* __restrict__ slots, g2_jac* __restrict__ h) {
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

// task_pk's first half for the latency path (k_prep_wide runs r * acc on point programs,
// bgv_tg1.h): the set's key sum into *acc and true when the multiplication remains, else the
// final status written and false.
static __device__ __noinline__ bool task_pk_sum(uint32_t s, const bgv_dslot* __restrict__ slots,
                                                const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                                const uint8_t* __restrict__ pk_bytes, int32_t* __restrict__ pk_status,
                                                const g1_jac* __restrict__ pk_agg, g1_jac* acc) {
  const bgv_dslot& d = slots[s];
  if (d.flags & BGV_SLOT_PAD) {
    pk_status[s] = BGV_ST_INFINITY;
    return false;
  }
  int32_t st = BGV_ST_OK;
  const g1_jac a = pk_sum(d, pk_idx, cache, pk_bytes, pk_agg, s, &st);
  if (st != BGV_OK || jac_is_inf(a)) {  // r * acc is infinity iff acc is (acc in G1, r != 0 mod r_G1)
    pk_status[s] = st != BGV_OK ? st : BGV_ST_INFINITY;
    return false;
  }
  *acc = a;
  return true;
}

static __device__ __noinline__ void task_pk(uint32_t s, const bgv_dslot* __restrict__ slots,
                                     const uint32_t* __restrict__ pk_idx, const g1_aff* __restrict__ cache,
                                     const uint8_t* __restrict__ pk_bytes, g1_jac* __restrict__ rpk,
                                     int32_t* __restrict__ pk_status, const g1_jac* __restrict__ pk_agg) {
  const bgv_dslot& d = slots[s];
  int32_t st = BGV_ST_OK;
  if (d.flags & BGV_SLOT_PAD) {
    pk_status[s] = BGV_ST_INFINITY;
    return;
  }
  const g1_jac acc = pk_sum(d, pk_idx, cache, pk_bytes, pk_agg, s, &st);
  if (st == BGV_OK) {
    // Jacobian: the Miller loop takes P projectively (bls_pairing.h miller_p), no inversion
    const g1_jac rp = jac_mul_glv(acc, d.scalar);
    if (jac_is_inf(rp))
      st = BGV_ST_INFINITY;  // infinity aggregate: BLST_PK_IS_INFINITY / false (job_precheck)
    else
      rpk[s] = rp;
  }
  pk_status[s] = st;
}

