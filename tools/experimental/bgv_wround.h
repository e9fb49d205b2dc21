// Round programs (bgv_tmiller.h / bgv_tcurve.h) on four wavefronts with wave-cooperative
// products (bgv_wfp.h layout: one limb per lane).
//
// The four-part engine (bgv_tround_dev.h) puts a round's 16 instructions on one wave, each lane
// computing a whole double-width product and its reduction: a round costs one product's ~500
// instructions of one wave plus the operand combinations and the part sum (2.4 us).  A round of
// the G2 point programs has only 4..10 real instructions (the rest write the DUMMY slot), so
// here each real instruction REDC(sum_k lin(A_k) lin(B_k)) runs on ONE wave with the limbs
// spread over the lanes, and the block's four waves (one per SIMD) take the instructions
// c = w, w + 4, ...: a round costs the longest wave's one or two instructions of ~250-320
// instructions each.
//
// Per instruction, limb l of every value in lane l (lanes >= 14 hold 0):
//   lin      K p_l + sum_j c_j S[j]_l as a signed 64-bit value per lane, two signed carry passes
//            (DPP wave_shr): digits in [-1, 2^28], the value unchanged (>= 0, < 2^392 by the
//            generator's bounds)
//   a.b      the 28 column sums of wfp_mul3 (lanes 50..63 columns 0..13, lanes 0..13 columns
//            14..27) with signed multiply-adds, summed over the T products
//   t        T mod R: three signed passes over the low lanes, then an exact resolution of the
//            digits (ballot carry lookahead; the carry out of column 13 dropped): t in [0, R)
//   m, U     m = t N' mod R (two passes, m < R (1 + 2^-19)), U = T + m p (wfp_umul's rotations)
//   out      three signed passes over the ring, the low half resolved exactly (its carry out,
//            0 or 1, into column 14), the high half resolved exactly: normalized limbs, the value
//            (ab + mp) / R -- the same integer as tmp_lane's wide_redc, so the same slot values.
#pragma once
#include "bgv_tcurve.h"
#include "bgv_wfp.h"

#if defined(__HIPCC__)

// lane L reads lane L - 1 of a 64-bit value (lane 0 reads 0)
__device__ __forceinline__ int64_t wr_shr64(int64_t v, uint32_t lane) {
  const uint32_t lo = wfp_shr1((uint32_t)v, lane), hi = wfp_shr1((uint32_t)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// lane L reads lane (L - 1) mod 64 of a 64-bit value
__device__ __forceinline__ int64_t wr_ror64(int64_t v) {
  const uint32_t lo = wfp_ror1((uint32_t)v), hi = wfp_ror1((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// one signed carry pass: digit = low 28 bits + the lower neighbour's arithmetic carry
__device__ __forceinline__ int64_t wr_pass(int64_t x, uint32_t lane) {
  return (x & (int64_t)LMASK) + wr_shr64(x >> LBITS, lane);
}
__device__ __forceinline__ int64_t wr_pass_ring(int64_t x) { return (x & (int64_t)LMASK) + wr_ror64(x >> LBITS); }

// Carry lookahead over the contiguous lane bits of `range`: generate G, propagate P (disjoint)
// -> bit i of the result = the carry into lane i; *top_out = the carry out of the top lane.
__device__ __forceinline__ uint64_t wr_carries(uint64_t G, uint64_t P, uint64_t range, bool* top_out) {
  G &= range;
  P &= range;
  const uint64_t X = G | P, S = X + G;
  const uint64_t C = S ^ X ^ G;  // bit i: carry into bit i (X + G, X = G | P, X & G = G, X ^ G = P)
  const uint64_t top = range & ~(range >> 1);
  *top_out = top == (1ull << 63) ? S < X : (C & (top << 1)) != 0;
  return C & range;
}

// Exact resolution of digits d in [-1, 2^28 + 1] over the lanes of `range` (contiguous): the
// positive carries first (generate d >= 2^28, propagate d == 2^28 - 1), then the borrows of
// the -1 digits (generate d == -1, propagate d == 0), each one 64-bit add of ballot masks.
// Returns the digit in [0, 2^28) (0 outside the range); *out (if given) receives the net carry
// out of the range's top lane (-1, 0 or 1).
__device__ __forceinline__ uint32_t wr_resolve(int64_t d, uint32_t lane, uint64_t range, int* out) {
  const bool in = (range >> lane) & 1;
  const bool is_top = in && !((range >> lane) & 2);
  bool top;
  uint64_t C = wr_carries(__ballot(in && d >= (int64_t)(1u << LBITS)), __ballot(in && d == (int64_t)LMASK), range, &top);
  const bool ci = (C >> lane) & 1;
  const bool co = is_top ? top : in && ((C >> (lane + 1)) & 1);
  const int64_t e = d + (ci ? 1 : 0) - (co ? (int64_t)(1u << LBITS) : 0);
  bool btop;
  C = wr_carries(__ballot(in && e < 0), __ballot(in && e == 0), range, &btop);
  const bool bi = (C >> lane) & 1;
  const bool bo = is_top ? btop : in && ((C >> (lane + 1)) & 1);
  const int64_t f = e - (bi ? 1 : 0) + (bo ? (int64_t)(1u << LBITS) : 0);
  if (out) *out = (top ? 1 : 0) - (btop ? 1 : 0);
  return in ? (uint32_t)f : 0u;
}

struct wr_ctx {
  uint32_t lane;
  int64_t p_lane;  // p's limb in lanes 0..13
};

__device__ __forceinline__ wr_ctx wr_init() {
  wr_ctx c;
  c.lane = wfp_lane();
  uint32_t r = 0;
  BGV_UNROLL for (int l = 0; l < NL; ++l) r = c.lane == (uint32_t)l ? p_limb(l) : r;
  c.p_lane = r;
  return c;
}

// lin(): K p + sum_j c_j S[idx_j], digits in [-1, 2^28] (signed 32-bit), lanes >= 14 zero
__device__ __forceinline__ int32_t wr_lin(const fp_t* S, const uint8_t* q, int M, const wr_ctx& c) {
  const bool live = c.lane < NL;
  int64_t acc = (int64_t)q[2 * M] * c.p_lane;
  for (int j = 0; j < M; ++j) {
    const int32_t cf = (int8_t)q[2 * j + 1];
    const int32_t x = live ? (int32_t)S[q[2 * j]].v[c.lane] : 0;
    acc += (int64_t)cf * x;
  }
  acc = wr_pass(wr_pass(acc, c.lane), c.lane);
  return live ? (int32_t)acc : 0;
}

// col += a * b over the 28 columns (signed digits)
__device__ __forceinline__ void wr_mac(int64_t& col, int32_t a, int32_t b) {
  int32_t br[NL];
  uint32_t r = (uint32_t)b;
  BGV_UNROLL for (int k = 1; k <= NL; ++k) {
    r = wfp_rol1(r);
    br[NL - k] = (int32_t)r;
  }
  BGV_UNROLL for (int i = NL - 1; i >= 0; --i)
    col += (int64_t)__builtin_amdgcn_readlane(a, i) * (int64_t)br[i];
}

// (col + m p) / R, normalized limbs in lanes 0..13 (value < 2p for the generator's bounds)
__device__ __forceinline__ uint32_t wr_reduce(int64_t col, const wr_ctx& c) {
  const uint32_t lane = c.lane;
  const uint64_t LOW = 0xFFFC000000000000ull, HIGH = 0x3FFFull;
  // t = col mod R in lanes 50..63
  const int64_t t2 = wr_pass(wr_pass(wr_pass(col, lane), lane), lane);  // |col| < 2^62: three passes
  const uint32_t t = wr_resolve(t2, lane, LOW, nullptr);
  const uint32_t NP[NL] = BGV_NPRIME_LIMBS;
  uint64_t M = (uint64_t)NP[0] * t;
  uint32_t tr = t;
  BGV_UNROLL for (int j = 1; j < NL; ++j) {
    tr = wfp_ror1(tr);
    M += (uint64_t)NP[j] * tr;
  }
  uint32_t m;
  {
    const uint64_t h = M >> LBITS;
    const uint64_t v1 = (uint64_t)((uint32_t)M & LMASK) +
                        (((uint64_t)wfp_shr1((uint32_t)(h >> 32), lane) << 32) | wfp_shr1((uint32_t)h, lane));
    m = ((uint32_t)v1 & LMASK) + wfp_shr1((uint32_t)(v1 >> LBITS), lane);
    m = lane >= 50 ? m : 0u;
  }
  uint32_t mr = m;
  int64_t U = col + (int64_t)((uint64_t)p_limb(0) * mr);
  BGV_UNROLL for (int j = 1; j < NL; ++j) {
    mr = wfp_ror1(mr);
    U += (int64_t)((uint64_t)p_limb(j) * mr);
  }
  U = wr_pass_ring(wr_pass_ring(wr_pass_ring(U)));
  int cl = 0;
  (void)wr_resolve(U, lane, LOW, &cl);  // the low half: a multiple of R, all digits 0 after it
  const int64_t hi = U + (lane == 0 ? (int64_t)cl : 0);
  return wr_resolve(hi, lane, HIGH, nullptr);
}

// one instruction of a round on the calling wave: REDC(sum_k lin(A_k) lin(B_k))
__device__ __forceinline__ uint32_t wr_instr(const fp_t* S, const uint8_t* rec, int T, int M, const wr_ctx& c) {
  int64_t col = 0;
  const uint8_t* q = rec + 1;
  for (int k = 0; k < T; ++k) {
    const int32_t a = wr_lin(S, q, M, c);
    const int32_t b = wr_lin(S, q + 2 * M + 1, M, c);
    wr_mac(col, a, b);
    q += 2 * (2 * M + 1);
  }
  return wr_reduce(col, c);
}

// The point-program engine of bgv_tcurve.h's schedules on a 256-thread block (four waves, one
// set): instruction c of a round on wave c % 4 (DUMMY instructions skipped), one block barrier
// per round (no slot is read and written in one round).  Bank moves by the first threads.
struct tc_wave4_engine {
  const uint8_t* prog;
  fp_t* S;
  wr_ctx cx;
  int w;     // wave 0..3
  bool bad;  // thread 0: an exceptional addition was met
  __device__ void run(int off) {
    int pos = off;
    const int nr = prog[pos++];
    for (int r = 0; r < nr; ++r) {
      const int T = prog[pos], M = prog[pos + 1];
      pos += 2;
      const int rb = tmp_rec_bytes(T, M);
      for (int ci = w; ci < BGV_TEAM; ci += 4) {
        const uint8_t* rec = prog + pos + ci * rb;
        const int out = rec[0];
        if (out == TCP_S_DUMMY) continue;
        const uint32_t v = wr_instr(S, rec, T, M, cx);
        if (cx.lane < NL) S[out].v[cx.lane] = v;
      }
      __syncthreads();
      pos += BGV_TEAM * rb;
    }
  }
  __device__ void copy(int dst, int src) {  // src may differ per block (a digit's table entry)
    const int t = threadIdx.x;
    if (dst != src && t < 6 * NL) S[TCP_BANK(dst) + t / NL].v[t % NL] = S[TCP_BANK(src) + t / NL].v[t % NL];
    __syncthreads();
  }
  __device__ void neg_y(int b) {
    const int t = threadIdx.x;
    if (t == 2 || t == 3) S[TCP_BANK(b) + t] = fp_neg(S[TCP_BANK(b) + t]);
    __syncthreads();
  }
  __device__ void check_add() {
    if (threadIdx.x == 0) {
      const auto z2 = [&](int s) { return fp_is_zero(S[s]) && fp_is_zero(S[s + 1]); };
      bad = bad || z2(TC_CHK_A) || z2(TC_CHK_B);
    }
  }
};

#endif  // __HIPCC__
