// The latency path's first per-set tasks (SSWU maps and signature decoding), shared by the
// latency-path unit (bgv_k_prep.hip: one lane per set) and the wave-uniform unit
// (bgv_k_prep_wave.hip: one set per wave, every product on the whole wave).
#pragma once
#include "bgv_k_tasks.h"

// ---- latency path ------------------------------------------------------------------------
// f[s] (576 B, written by k_miller only later) holds the split's intermediates:
// q1 = the u1 map's point (g2_jac, 288 B) at offset 0, the decoded signature (g2_aff) at 288.
static __device__ __forceinline__ g2_jac* split_q1(fp12_t* f, uint32_t s) { return reinterpret_cast<g2_jac*>(f + s); }
static __device__ __forceinline__ g2_aff* split_sig(fp12_t* f, uint32_t s) {
  return reinterpret_cast<g2_aff*>(reinterpret_cast<uint8_t*>(f + s) + sizeof(g2_jac));
}
static_assert(sizeof(g2_jac) + sizeof(g2_aff) <= sizeof(fp12_t), "split intermediates fit in f[s]");

// one of the two SSWU maps of hash_to_G2 (bls_hash.h hash_to_g2), the point on E2' (Jacobian):
// the 3-isogeny runs in the next launch's point programs (tools/gen_tcurve.py iso12_45).
// PW: the square roots' exponentiations on this lane (bgv_pow_lane) or on the whole wave
// (bgv_pow_wave, one set per wave, every lane computing the same values; lane 0 writes).
template <class PW>
__device__ __noinline__ void task_map_t(uint32_t s, int which, const bgv_dslot* __restrict__ slots, g2_jac* out,
                                        bool writer) {
  const bgv_dslot& d = slots[s];
  if (d.flags & BGV_SLOT_PAD) return;
  uint8_t msg[32];
  for (int i = 0; i < 32; ++i) msg[i] = d.msg[i];
  fp2_t u0, u1;
  hash_to_field_fp2(&u0, &u1, msg, 32);
  const g2_jac q = sswu_g2_jac_t<PW>(which ? u1 : u0, fp_sqrt_minus5());
  if (writer) *out = q;
}

// task_sig's decoding half: status, and the affine point when it decodes to a finite point
template <class PW>
__device__ __noinline__ void task_sig_decode_t(uint32_t s, const bgv_dslot* __restrict__ slots, g2_aff* out,
                                               int32_t* __restrict__ sig_status, bool writer) {
  const bgv_dslot& d = slots[s];
  int32_t st = BGV_ST_OK;
  g2_aff a;
  bool fin = false;
  if (d.flags & BGV_SLOT_PAD) {
    st = BGV_ST_INFINITY;
  } else if (d.sig_len != 96) {
    st = BGV_INVALID_SIZE;
  } else {
    uint8_t b[96];
    for (int i = 0; i < 96; ++i) b[i] = d.sig[i];
    bool inf;
    st = g2_decompress_t<PW>(&a, &inf, b);
    if (st == BGV_OK) {
      if (inf)
        st = BGV_ST_INFINITY;
      else
        fin = true;
    }
  }
  if (writer) {
    if (fin) *out = a;
    sig_status[s] = st;
  }
}

