// The generated point programs (bgv_tcurve_prog.h: rounds of instructions REDC(sum_k lin(A_k)
// lin(B_k)), tools/gen_tcurve.py) in residue arithmetic (bgv_rns.h), for the latency path's G2
// scalar multiplications (k_prep_wide: the cofactor clearing, r * sig, [|x|]P).
//
// A 512-thread block (eight waves) holds the program's slots as 30 residues each (LDS
// [slot][32]); instruction c of a round runs on the 30-lane group c (two per wave), every lane
// evaluating its residue of the instruction's linear forms and products lane-locally, then ONE
// Montgomery reduction of the sum (two base extensions inside the wave) -- against the
// four-part engine (bgv_tround_dev.h), where a lane waits one double-width 14 x 14 product, a
// 14-row reduction and two carry-chained linear forms per round.  One block barrier per round.
// A negative coefficient takes the slot as 16p - X (slots hold integers X <= 16p), so every
// linear form is a non-negative integer below 16p sum |c_j| and every product sum stays far
// below M p (bgv_rns.h's bound); the generator's K p terms (for 28-bit limbs below 2p) are not
// needed.  The values are the same field elements as the four-part engine's (every instruction
// is the same product of the same linear forms mod p), in the RNS Montgomery form x M.
#pragma once
#include "bgv_rns.h"
#include "bgv_tcurve.h"

#define BGV_RNS_ROUND_THREADS 512
#define BGV_RNS_ROUND_INSTR 16  // instructions per round (the programs' team width)
static_assert(BGV_RNS_ROUND_THREADS / 32 == BGV_RNS_ROUND_INSTR, "one 30-lane group per instruction");

struct rns_round_engine : rns_lane {
  const uint8_t* prog;
  uint32_t (*S)[32];  // the slots
  bool bad;

  __device__ void init(uint32_t (*slots)[32], rns_xch* x, const uint8_t* p, int tid) {
    lane_init(x, tid);
    S = slots;
    prog = p;
    bad = false;
  }
  // this lane's residue of sum_j c_j X_j, negative c_j as |c_j| (16p - X_j)
  // a linear form's residue sum (< 2^28 M 128) folded once: below 2^29, a product operand
  __device__ __forceinline__ uint32_t fold(uint64_t a) const { return (uint32_t)(a >> 28) * c1 + ((uint32_t)a & 0xfffffffu); }
  template <int M>
  __device__ __forceinline__ uint32_t lin(const uint8_t* q) const {
    uint64_t acc = 0;
    BGV_UNROLL for (int j = 0; j < M; ++j) {
      const uint32_t x = S[q[2 * j]][i];
      const int cf = (int8_t)q[2 * j + 1];
      acc += (uint64_t)(uint32_t)(cf < 0 ? -cf : cf) * (cf < 0 ? negm(x) : x);
    }
    return fold(acc);
  }
  __device__ uint32_t lin_any(const uint8_t* q, int M) const {
    uint64_t acc = 0;
    for (int j = 0; j < M; ++j) {
      const uint32_t x = S[q[2 * j]][i];
      const int cf = (int8_t)q[2 * j + 1];
      acc += (uint64_t)(uint32_t)(cf < 0 ? -cf : cf) * (cf < 0 ? negm(x) : x);
    }
    return fold(acc);
  }
  template <int T, int M>
  __device__ __forceinline__ uint32_t instr(const uint8_t* rec) const {
    uint64_t acc = 0;
    BGV_UNROLL for (int k = 0; k < T; ++k) {
      const uint8_t* q = rec + 1 + k * 2 * (2 * M + 1);
      acc += (uint64_t)lin<M>(q) * lin<M>(q + 2 * M + 1);
    }
    return red(acc);
  }
  __device__ uint32_t instr_any(const uint8_t* rec, int T, int M) const {
    switch (T * 8 + M) {  // the shapes the generated tables use (bgv_tmiller.h tmp_lane_any)
      case 1 * 8 + 1: return instr<1, 1>(rec);
      case 1 * 8 + 4: return instr<1, 4>(rec);
      case 2 * 8 + 1: return instr<2, 1>(rec);
      case 2 * 8 + 2: return instr<2, 2>(rec);
      case 2 * 8 + 4: return instr<2, 4>(rec);
      case 3 * 8 + 4: return instr<3, 4>(rec);
      case 4 * 8 + 2: return instr<4, 2>(rec);
      case 4 * 8 + 3: return instr<4, 3>(rec);
      default: {
        uint64_t acc = 0;
        for (int k = 0; k < T; ++k) {
          const uint8_t* q = rec + 1 + k * 2 * (2 * M + 1);
          acc += (uint64_t)lin_any(q, M) * lin_any(q + 2 * M + 1, M);
        }
        return red(acc);
      }
    }
  }
  // the rounds of the program at off; every thread of the block must call it
  __device__ void run(int off) {
    int pos = off;
    const int nr = prog[pos++];
    for (int r = 0; r < nr; ++r) {
      const int T = prog[pos], M = prog[pos + 1];
      pos += 2;
      const int rb = tmp_rec_bytes(T, M);
      const uint8_t* rec = prog + pos + g * rb;
      const uint32_t v = mont(live ? instr_any(rec, T, M) : 0u);
      // no slot is read and written in one round (the generators check it): no barrier before
      if (live) S[rec[0]][i] = v;
      __syncthreads();
      pos += BGV_RNS_ROUND_INSTR * rb;
    }
  }
  // fp_t values (28-bit, R form) into slots: value k on group k (k < n <= 16); all threads call
  __device__ void put(const int* slot, const fp_t* v, int n) {
    const uint32_t r = from_fp(g < n ? v[g] : fp_zero());
    if (g < n && live) S[slot[g]][i] = r;
    __syncthreads();
  }
  // slots back to fp_t (valid in out[] after the call); all threads call
  __device__ void get(const int* slot, fp_t* out, int n) {
    const fp_t r = to_fp(g < n && live ? S[slot[g]][i] : 0u);
    if (g < n && i == 0) out[g] = r;
    __syncthreads();
  }
};

// bgv_tcurve.h's engine interface over the six-slot G2 banks
struct rns_tc_engine : rns_round_engine {
  __device__ void copy(int dst, int src) {
    if (dst != src && g < 6 && live) S[TCP_BANK(dst) + g][i] = S[TCP_BANK(src) + g][i];
    __syncthreads();
  }
  __device__ void neg_y(int b) {
    if (g < 2 && live) S[TCP_BANK(b) + 2 + g][i] = negm(S[TCP_BANK(b) + 2 + g][i]);
    __syncthreads();
  }
  // an exceptional addition: v^2 or Z1 Z2 (Fp2) zero
  __device__ void check_add() {
    if (threadIdx.x < 4) X->zm[threadIdx.x] = 0x1ffffu;
    __syncthreads();
    if (g < 4 && live) atomicAnd(&X->zm[g], zero_mask(S[g < 2 ? TC_CHK_A + g : TC_CHK_B + g - 2][i]));
    __syncthreads();
    bad = bad || (X->zm[0] && X->zm[1]) || (X->zm[2] && X->zm[3]);
    __syncthreads();
  }
  // the constant slots of every schedule (one, psi's and psi^2's coefficients, the isogeny's)
  __device__ void init_consts() {
    const fp2_t cx = BGV_PSI_CX, cy = BGV_PSI_CY;
    const fp_t c0[7] = {fp_one(), cx.c0, cx.c1, cy.c0, cy.c1, fp_t{BGV_PSI2_CX}, fp_t{BGV_PSI2_CY}};
    const int s0[7] = {TCP_S_ONE, TCP_S_PSI_CX, TCP_S_PSI_CX + 1, TCP_S_PSI_CY, TCP_S_PSI_CY + 1, TCP_S_PSI2_CX,
                       TCP_S_PSI2_CY};
    put(s0, c0, 7);
    for (int b = 0; b < TC_ISO_NCONST; b += BGV_RNS_ROUND_INSTR) {
      const int n = TC_ISO_NCONST - b < BGV_RNS_ROUND_INSTR ? TC_ISO_NCONST - b : BGV_RNS_ROUND_INSTR;
      fp_t v[BGV_RNS_ROUND_INSTR];
      int s[BGV_RNS_ROUND_INSTR];
      BGV_UNROLL for (int k = 0; k < BGV_RNS_ROUND_INSTR; ++k) {
        v[k] = k < n ? tc_iso_const(b + k) : fp_zero();
        s[k] = TCP_S_ISO + b + k;
      }
      put(s, v, n);
    }
  }
};
