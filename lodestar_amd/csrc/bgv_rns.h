// Residue-number-system Fp12 engine for the latency path (gfx950): one Fp12 value spread over
// 12 x 30 lanes of a 384-thread block, each lane holding ONE residue of ONE Fp coefficient.
//
// An Fp element is an integer X < 16p (X = x M mod p: RNS Montgomery form) kept as its residues
// modulo 30 primes m = 2^28 - c (base B: lanes i < 15, product M ~ 2^420; base B': i = 15..29).
// Lane (c, i) of wave w: coefficient c = 2w + (lane >> 5) (w-basis, c = 2k + e as bls_team.h),
// residue i = lane & 31 (i = 30, 31 idle).  An Fp12 product is then:
//   1. lane-local: the 12 products of coefficient c (bls_team.h tm_mul_lane's terms, negation as
//      16p - x) summed in 64 bits and reduced mod m -- the whole double-width coefficient;
//   2. ONE Montgomery reduction per coefficient (Bajard / Kawamura): q = -s p^-1 mod M on the B
//      lanes, extended to B' (fast extension, q^ = q + alpha M), r = (s + q^ p) / M on the B'
//      lanes, extended back to B exactly (alpha from a fixed-point sum, exact since r < M' 2^-34).
//      Each extension is a 15-term dot product per lane over the other half's values, exchanged
//      through LDS inside the wave (both halves of a coefficient share a wave: no block barrier).
// One block barrier per operation (the next operation's operands come from every wave).
// Against the eight-part team products (bls_team.h tm_*_part8: a lane waits 1-2 double-width
// 14x14 products plus a 14-row reduction) a lane here waits ~12 + 2 x 15 single-word products.
// Constants: bgv_rns_consts.h (tools/gen_rns.py, which also models these lanes exactly and
// checks them against big integers and the oracle's Fp12 products).
#pragma once
#include "bls_team.h"
#include "bgv_rns_consts.h"

#define BGV_RNS_THREADS 384  // the Fp12 engine: 12 coefficients, two per wave
#define BGV_RNS_GROUPS 16    // 30-lane groups an engine may have (the round engine: 16, eight waves)

// The exchange area of the reductions, one row per 30-lane group (g = 2 wave + half)
struct rns_xch {
  uint32_t x[BGV_RNS_GROUPS][16];     // the B lanes' xi of a reduction
  uint32_t xp[BGV_RNS_GROUPS][16];    // the B' lanes' xi'
  long long col[BGV_RNS_GROUPS][16];  // to_fp: the integer's 28-bit columns
  uint32_t zm[BGV_RNS_GROUPS];        // zero tests: per group, the AND of the lanes' masks
};

__device__ __forceinline__ void rns_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// One lane's residue arithmetic: group g (the 30 lanes holding one Fp value), residue i.
struct rns_lane {
  rns_xch* X;
  int g, i;
  bool live, isb;  // i < 30; i < 15
  uint32_t m, c1, c16, xi, xi2, aux, pm, kp;
  uint32_t row[BGV_RNS_NB];

  __device__ void lane_init(rns_xch* x, int tid) {
    X = x;
    const int w = tid >> 6, l = tid & 63;
    g = 2 * w + (l >> 5);
    i = l & 31;
    live = i < BGV_RNS_NL;
    isb = i < BGV_RNS_NB;
    const int ii = live ? i : 0;
    m = kRnsMod[ii];
    c1 = (1u << 28) - m;
    c16 = 16u * c1;
    xi = kRnsXi[ii];
    xi2 = kRnsXi2[ii];
    aux = kRnsAux[ii];
    pm = kRnsPm[ii];
    kp = kRnsKp[ii];
    BGV_UNROLL for (int j = 0; j < BGV_RNS_NB; ++j) row[j] = kRnsRow[ii * BGV_RNS_NB + j];
  }
  // x < 2^64 -> x mod m: 2^32 = 16 c, then 2^28 = c (mod m)
  __device__ __forceinline__ uint32_t red(uint64_t x) const {
    const uint64_t y = (uint64_t)(uint32_t)(x >> 32) * c16 + (uint32_t)x;
    const uint64_t z = (uint64_t)(uint32_t)(y >> 32) * c16 + (uint32_t)y;
    const uint32_t w = (uint32_t)(z >> 28) * c1 + ((uint32_t)z & 0xfffffffu);
    const uint32_t d = w - m;
    return d < w ? d : w;  // w < 2m
  }
  __device__ __forceinline__ uint32_t mulm(uint32_t a, uint32_t b) const { return red((uint64_t)a * b); }
  // 16p - x (x < 16p as an integer): the negation every form here uses
  __device__ __forceinline__ uint32_t negm(uint32_t a) const {
    const uint32_t t = kp + (m - a);
    const uint32_t d = t - m;
    return d < t ? d : t;
  }
  // bit t set iff this residue is that of t p (t <= 16): an integer X <= 16p is 0 mod p iff the
  // AND of its 30 lanes' masks is nonzero (X and t p < M, CRT)
  __device__ uint32_t zero_mask(uint32_t a) const {
    uint32_t mask = 0, v = 0;
    BGV_UNROLL for (int t = 0; t <= BGV_RNS_KNEG; ++t) {
      mask |= (a == v ? 1u : 0u) << t;
      const uint32_t u = v + pm, d = u - m;
      v = d < u ? d : u;
    }
    return mask;
  }

  // one Montgomery reduction of this lane's coefficient: s -> s M^-1 (mod p), < 16p
  __device__ uint32_t mont(uint32_t s) {
    uint32_t r = 0;
    if (isb) X->x[g][i] = mulm(s, xi);
    rns_wave_sync();
    if (live && !isb) {
      // independent partial sums (one per quad of xi): the chains of dependent 64-bit
      // multiply-adds are the latency here, not their count
      const uint4* Q = reinterpret_cast<const uint4*>(X->x[g]);
      uint64_t a4[4];
      BGV_UNROLL for (int q = 0; q < 4; ++q) {
        const uint4 v = Q[q];
        uint64_t a = (uint64_t)v.x * row[4 * q];
        a += (uint64_t)v.y * row[4 * q + 1];
        a += (uint64_t)v.z * row[4 * q + 2];
        if (4 * q + 3 < BGV_RNS_NB) a += (uint64_t)v.w * row[4 * q + 3];
        a4[q] = a;
      }
      const uint32_t qh = red((a4[0] + a4[1]) + (a4[2] + a4[3]));
      const uint32_t t = red((uint64_t)qh * pm + s);       // s + q^ p
      r = mulm(t, aux);                                      // (s + q^ p) M^-1
      X->xp[g][i - BGV_RNS_NB] = mulm(t, xi2);               // r M'_j^-1, beside r
    }
    rns_wave_sync();
    if (isb) {
      const uint4* Q = reinterpret_cast<const uint4*>(X->xp[g]);
      uint64_t a2[2] = {0, 0}, b2[2] = {BGV_RNS_BETA_ROUND, 0};
      BGV_UNROLL for (int q = 0; q < 4; ++q) {
        const uint4 v = Q[q];
        const uint32_t t[4] = {v.x, v.y, v.z, v.w};
        BGV_UNROLL for (int z = 0; z < 4; ++z) {
          const int j = 4 * q + z;
          if (j >= BGV_RNS_NB) continue;
          a2[q & 1] += (uint64_t)t[z] * row[j];
          b2[q & 1] += (uint64_t)t[z] * kRnsGBeta[j];
        }
      }
      const uint32_t beta = (uint32_t)((b2[0] + b2[1]) >> BGV_RNS_BETA_SHIFT);
      r = red((a2[0] + a2[1]) + (uint64_t)beta * aux);  // - beta M'
    }
    return r;
  }

  // fp_t (28-bit limbs, Montgomery R = 2^392, < 2p) -> this lane's residue of x M
  __device__ uint32_t from_fp(const fp_t& x) {
    uint32_t s = 0;
    if (live) {
      uint64_t acc = 0;
      BGV_UNROLL for (int q = 0; q < NL; ++q) acc += (uint64_t)x.v[q] * kRnsL28[i * 15 + q];
      s = mulm(red(acc), kRnsCin[i]);  // x R * (M^2 / R) -> mont -> x M
    }
    return mont(s);
  }
  // this lane's coefficient back to an fp_t (R = 2^392 form, < 2p), valid on the lanes i == 0:
  // z = x R as an integer < 16p (one product by R mod p), then z = sum_i xi_i M_i - beta M over
  // base B (xi_i = z_i M_i^-1 mod m_i, beta exact as in mont) in 28-bit columns, one lane per
  // column, and the carries on lane 0.  Every lane of the block must call it.
  __device__ fp_t to_fp(uint32_t a) {
    const uint32_t z = mont(live ? mulm(a, kRnsCout[i]) : 0u);
    if (isb) X->x[g][i] = mulm(z, kRnsMinvB[i]);
    rns_wave_sync();
    if (i < 16) {
      uint64_t acc = 0, bacc = BGV_RNS_BETA_ROUND;
      BGV_UNROLL for (int j = 0; j < BGV_RNS_NB; ++j) {
        const uint32_t x = X->x[g][j];
        if (i < 15) acc += (uint64_t)x * kRnsMiLimbs[j * 15 + i];
        bacc += (uint64_t)x * kRnsGB[j];
      }
      const uint32_t beta = (uint32_t)(bacc >> BGV_RNS_BETA_SHIFT);
      X->col[g][i] = (long long)acc - (long long)((uint64_t)beta * kRnsMLimbs[i]);
    }
    rns_wave_sync();
    fp_t r = fp_zero();
    if (i == 0) {
      lz<LMASK, BGV_RNS_KNEG> t;
      long long cy = 0;
      // 16 columns (M_i and M reach bits 392..419); the value < 16p < 2^385 leaves limbs
      // 14 and 15 zero and limb 13 below 2^21
      BGV_UNROLL for (int q = 0; q < 16; ++q) {
        const long long v = X->col[g][q] + cy;
        if (q < NL) t.v[q] = (uint32_t)(v & LMASK);
        cy = v >> LBITS;
      }
      r = lz_out(t);
    }
    return r;
  }
};

// The Fp12 engine (tm_final_exp_u's operations over E = this lane's residue): coefficient c =
// the lane's group (w-basis, c = 2k + e), six waves.
struct rns_smem {
  uint32_t v[2][12][32];  // operand a (two buffers: operation n + 1 writes while n is read)
  uint32_t w[2][12][32];  // operand b
  rns_xch xch;
};

struct rns_ops : rns_lane {
  rns_smem* S;
  int c, k, e;  // coefficient (= g), w-power, real/imaginary
  int buf;
  __device__ void init(rns_smem* s, int tid) {
    S = s;
    lane_init(&s->xch, tid);
    c = g;
    k = c >> 1;
    e = c & 1;
    buf = 0;
  }
  // the unreduced coefficient (k, e) of a * b from the operand buffers A, B
  __device__ uint32_t prod(const uint32_t (*A)[32], const uint32_t (*B)[32]) const {
    uint64_t acc = 0, acc2 = 0;  // two chains
    const uint32_t km = kp + m;
    BGV_UNROLL for (int ii = 0; ii < 6; ++ii) {
      const bool wrap = ii > k;
      const int j = wrap ? k + 6 - ii : k - ii;
      const uint32_t x0 = A[2 * ii][i], x1 = A[2 * ii + 1][i];
      const uint32_t y0 = B[2 * j][i], y1 = B[2 * j + 1][i];
      const uint32_t d = y0 + (km - y1), s = y0 + y1, x1n = km - x1;
      const uint32_t X2 = e ? x1 : x1n;
      const uint32_t Y1 = wrap ? (e ? s : d) : (e ? y1 : y0);
      const uint32_t Y2 = wrap ? (e ? d : s) : (e ? y0 : y1);
      acc += (uint64_t)x0 * Y1;
      acc2 += (uint64_t)X2 * Y2;
    }
    return red(acc + acc2);
  }

  __device__ uint32_t mul(uint32_t a, uint32_t b) {
    if (live) {
      S->v[buf][c][i] = a;
      S->w[buf][c][i] = b;
    }
    __syncthreads();
    const uint32_t s = live ? prod(S->v[buf], S->w[buf]) : 0u;
    buf ^= 1;
    return mont(s);
  }
  __device__ uint32_t sqr(uint32_t a) {
    if (live) S->v[buf][c][i] = a;
    __syncthreads();
    const uint32_t s = live ? prod(S->v[buf], S->v[buf]) : 0u;
    buf ^= 1;
    return mont(s);
  }
  // odd w-powers negated (16p - x)
  __device__ uint32_t conj(uint32_t a) const { return (k & 1) ? negm(a) : a; }
  // x -> x^p: conj(x_k) gamma_k, (x0 - x1 u)(g0 + g1 u) = (x0 g0 + x1 g1) + (x0 g1 - x1 g0) u
  __device__ uint32_t frob(uint32_t a) {
    if (live) S->v[buf][c][i] = a;
    __syncthreads();
    uint32_t s = 0;
    if (live) {
      const uint32_t x0 = S->v[buf][2 * k][i], x1 = S->v[buf][2 * k + 1][i];
      const uint32_t g0 = kRnsFrob1[(2 * k) * BGV_RNS_NL + i], g1 = kRnsFrob1[(2 * k + 1) * BGV_RNS_NL + i];
      const uint32_t x1n = kp + m - x1;
      s = e ? red((uint64_t)x0 * g1 + (uint64_t)x1n * g0) : red((uint64_t)x0 * g0 + (uint64_t)x1 * g1);
    }
    buf ^= 1;
    return mont(s);
  }
  // x -> x^(p^2): x_k gamma2_k (gamma2_k in Fp)
  __device__ uint32_t frob2(uint32_t a) {
    const uint32_t s = live ? mulm(a, kRnsFrob2[k * BGV_RNS_NL + i]) : 0u;
    return mont(s);
  }
  // every odd-w-power coefficient is 0 mod p: X in {0, p, ..., 16p} iff every residue matches
  // one t p for a common t (X, t p < M)
  __device__ bool is_fp6(uint32_t a) {
    if (threadIdx.x < 12) X->zm[threadIdx.x] = 0x1ffffu;
    __syncthreads();
    if (live && (k & 1)) atomicAnd(&X->zm[c], zero_mask(a));
    __syncthreads();
    const bool ok = X->zm[2] && X->zm[3] && X->zm[6] && X->zm[7] && X->zm[10] && X->zm[11];
    __syncthreads();
    return ok;
  }

};
