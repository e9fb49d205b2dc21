// hash_to_G2 on CDNA4: RFC 9380 suite BLS12381G2_XMD:SHA-256_SSWU_RO_, one
// message per lane.  SHA-256 (expand_message_xmd) -> hash_to_field (4 x Fp)
// -> 2 x simplified SWU on E2' -> 3-isogeny (Jacobian, no inversion) -> add
// -> clear_cofactor (psi method, RFC 9380 G.4).
#pragma once
#include "bls_curve.h"

// ---------------------------------------------------------------------------
// SHA-256
// ---------------------------------------------------------------------------
BGV_HD uint32_t sha_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

BGV_NOINLINE void sha256_compress(uint32_t st[8], const uint32_t blk[16]) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t w[16];
  BGV_UNROLL for (int i = 0; i < 16; ++i) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  BGV_UNROLL for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint32_t s0 = sha_rotr(w15, 7) ^ sha_rotr(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = sha_rotr(w2, 17) ^ sha_rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = sha_rotr(e, 6) ^ sha_rotr(e, 11) ^ sha_rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + K[i] + wi;
    uint32_t S0 = sha_rotr(a, 2) ^ sha_rotr(a, 13) ^ sha_rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

BGV_HD void sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u;
  st[1] = 0xbb67ae85u;
  st[2] = 0x3c6ef372u;
  st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu;
  st[5] = 0x9b05688cu;
  st[6] = 0x1f83d9abu;
  st[7] = 0x5be0cd19u;
}

// Hash a "virtual" message of total_len bytes whose byte at position i is
// get(i) (lane-uniform length, so every lane runs the same number of blocks).
template <class G>
BGV_HD void sha256_virtual(uint32_t out[8], const G& get, uint32_t total_len) {
  uint32_t st[8];
  sha256_init(st);
  const uint32_t padded = ((total_len + 9 + 63) / 64) * 64;
  const uint64_t bitlen = (uint64_t)total_len * 8;
  BGV_NO_UNROLL for (uint32_t base = 0; base < padded; base += 64) {
    uint32_t blk[16];
    BGV_UNROLL for (int wi = 0; wi < 16; ++wi) {
      uint32_t word = 0;
      BGV_UNROLL for (int k = 0; k < 4; ++k) {
        const uint32_t pos = base + (uint32_t)(wi * 4 + k);
        uint32_t byte;
        if (pos < total_len)
          byte = get(pos);
        else if (pos == total_len)
          byte = 0x80;
        else if (pos >= padded - 8)
          byte = (uint32_t)(bitlen >> (8 * (padded - 1 - pos))) & 0xff;
        else
          byte = 0;
        word = (word << 8) | byte;
      }
      blk[wi] = word;
    }
    sha256_compress(st, blk);
  }
  BGV_UNROLL for (int i = 0; i < 8; ++i) out[i] = st[i];
}

BGV_HD uint32_t dst_byte(uint32_t i) {
  // BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_ || I2OSP(43, 1)
  const char d[] = BGV_DST_POP;
  return i < BGV_DST_POP_LEN ? (uint32_t)(uint8_t)d[i] : (uint32_t)BGV_DST_POP_LEN;
}

struct xmd_b0_getter {
  const uint8_t* msg;
  uint32_t len;
  // Z_pad(64) || msg || I2OSP(256, 2) || 0x00 || DST_prime
  BGV_HD uint32_t operator()(uint32_t pos) const {
    if (pos < 64) return 0;
    pos -= 64;
    if (pos < len) return msg[pos];
    pos -= len;
    if (pos == 0) return 0x01;
    if (pos == 1) return 0x00;
    if (pos == 2) return 0x00;
    return dst_byte(pos - 3);
  }
};

struct xmd_bi_getter {
  const uint32_t* x;  // 8 words (b0 ^ b_{i-1})
  uint32_t idx;
  BGV_HD uint32_t operator()(uint32_t pos) const {
    if (pos < 32) return (x[pos >> 2] >> (24 - 8 * (pos & 3))) & 0xff;
    if (pos == 32) return idx;
    return dst_byte(pos - 33);
  }
};

// expand_message_xmd(msg, DST_POP, 256) -> 64 big-endian words
BGV_HD void expand_message_xmd_256(uint32_t ub[64], const uint8_t* msg, uint32_t len) {
  uint32_t b0[8], bi[8], x[8];
  xmd_b0_getter g0{msg, len};
  sha256_virtual(b0, g0, 64 + len + 3 + BGV_DST_POP_LEN + 1);
  BGV_UNROLL for (int k = 0; k < 8; ++k) x[k] = b0[k];
  BGV_NO_UNROLL for (uint32_t i = 1; i <= 8; ++i) {
    xmd_bi_getter gi{x, i};
    sha256_virtual(bi, gi, 32 + 1 + BGV_DST_POP_LEN + 1);
    BGV_UNROLL for (int k = 0; k < 8; ++k) {
      // store b_i: dynamic word index (i-1)*8+k; write via unrolled select to stay in registers
      x[k] = b0[k] ^ bi[k];
    }
    BGV_UNROLL for (int j = 1; j <= 8; ++j) {
      if (i == (uint32_t)j) {
        BGV_UNROLL for (int k = 0; k < 8; ++k) ub[(j - 1) * 8 + k] = bi[k];
      }
    }
  }
}

// bits [lo, lo+28) of a big-endian string of 16 u32 words (64 bytes)
BGV_HD uint32_t be_words_bits28(const uint32_t* w, int lo) {
  const int wi = lo >> 5, sh = lo & 31;  // word index from the little end
  uint64_t v = w[15 - wi];
  if (wi + 1 < 16) v |= (uint64_t)w[14 - wi] << 32;
  return (uint32_t)(v >> sh) & LMASK;
}

// 64 big-endian bytes (as 16 words) -> Fp (Montgomery), reduced mod p:
// value = hi * 2^392 + lo  ->  lo * R + hi * R^2 = mont(lo, R^2) + mont(hi, R^3)
BGV_HD fp_t fp_from_be64_words(const uint32_t* w) {
  fp_t lo, hi = fp_zero();
  BGV_UNROLL for (int i = 0; i < NL; ++i) lo.v[i] = be_words_bits28(w, LBITS * i);
  BGV_UNROLL for (int i = 0; i < 5; ++i) hi.v[i] = be_words_bits28(w, 392 + LBITS * i);
  hi.v[4] &= (1u << (512 - 392 - 4 * LBITS)) - 1;
  const fp_t r2 = {BGV_R2}, r3 = {BGV_R3};
  return fp_add(fp_mul(lo, r2), fp_mul(hi, r3));
}

BGV_HD void hash_to_field_fp2(fp2_t* u0, fp2_t* u1, const uint8_t* msg, uint32_t len) {
  uint32_t ub[64];
  expand_message_xmd_256(ub, msg, len);
  u0->c0 = fp_from_be64_words(ub + 0);
  u0->c1 = fp_from_be64_words(ub + 16);
  u1->c0 = fp_from_be64_words(ub + 32);
  u1->c1 = fp_from_be64_words(ub + 48);
}

// ---------------------------------------------------------------------------
// Simplified SWU on E2': y^2 = x^3 + A'x + B', A' = 240i, B' = 1012(1+i), Z = -(2+i)
// ---------------------------------------------------------------------------
// sqrt(-5) in Fp (Montgomery), used to turn sqrt(-n) into sqrt(N(Z) n), N(Z) = 5.
BGV_HD fp_t fp_sqrt_minus5() { return fp_t{BGV_SQRT_M5}; }

// If g is a square in Fp2: *y = sqrt(g), returns true.  Otherwise *y = sqrt(Z g).
// Two Fp exponentiations total (norm root + the Fp2 root).
BGV_NOINLINE bool fp2_sqrt_or_z(fp2_t* y, const fp2_t& g, const fp_t& sqrt_m5) {
  const fp2_t Z = BGV_SSWU_Z;
  const fp_t n = fp_add(fp_sqr(g.c0), fp_sqr(g.c1));
  const fp_t e = fp_pow_p_minus_3_div_4(n);
  const fp_t ne = fp_mul(n, e);
  const fp_t s = fp_mul(ne, e);
  const bool is_sq = fp_eq(s, fp_one()) || fp_is_zero(n);
  const fp2_t h = fp2_select(is_sq, fp2_mul(Z, g), g);
  const fp_t gam = fp_select(is_sq, fp_mul(sqrt_m5, fp_neg(ne)), ne);
  const bool h1z = fp_is_zero(h.c1);
  fp_t d = fp_select(h1z, fp_half(fp_add(h.c0, gam)), h.c0);
  fp_t t = fp_pow_p_minus_3_div_4(d);
  fp_t dt = fp_mul(d, t);
  fp_t s2 = fp_mul(dt, t);
  fp_t a1t2 = fp_half(fp_mul(h.c1, t));
  const bool qr = fp_eq(s2, fp_one());
  y->c0 = fp_select(qr, a1t2, dt);
  y->c1 = fp_select(qr, fp_neg(dt), a1t2);
  return is_sq;
}

// SWU on E2' in two halves so that two maps can share one inversion (Montgomery's trick):
// sswu_den gives den = Z^2 u^4 + Z u^2 (and Z u^2), sswu_finish takes 1/den (any value when
// den == 0: the exceptional case uses x1 = B / (Z A) and never reads it).
BGV_HD fp2_t sswu_den(const fp2_t& u, fp2_t* zu2) {
  const fp2_t Z = BGV_SSWU_Z;
  *zu2 = fp2_mul(Z, fp2_sqr(u));
  return fp2_add(fp2_sqr(*zu2), *zu2);
}

BGV_NOINLINE void sswu_finish(fp2_t* xo, fp2_t* yo, const fp2_t& u, const fp2_t& zu2, const fp2_t& den,
                              const fp2_t& den_inv, const fp_t& sqrt_m5) {
  const fp2_t A = BGV_SSWU_A, B = BGV_SSWU_B;
  const fp2_t bza = BGV_SSWU_B_OVER_ZA, mba = BGV_SSWU_MINUS_B_OVER_A;
  const bool den0 = fp2_is_zero(den);
  fp2_t x1 = fp2_mul(mba, fp2_add(fp2_one(), den_inv));
  x1 = fp2_select(den0, x1, bza);
  fp2_t gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
  fp2_t r;
  const bool sq = fp2_sqrt_or_z(&r, gx1, sqrt_m5);
  // non-square branch: x2 = Z u^2 x1, y = Z u^3 sqrt(Z gx1)
  fp2_t x2 = fp2_mul(zu2, x1);
  fp2_t y2 = fp2_mul(fp2_mul(zu2, u), r);
  fp2_t x = fp2_select(sq, x2, x1);
  fp2_t y = fp2_select(sq, y2, r);
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  *xo = x;
  *yo = y;
}

// returns the SWU point on E2' in affine coordinates
BGV_NOINLINE void sswu_g2(fp2_t* xo, fp2_t* yo, const fp2_t& u, const fp_t& sqrt_m5) {
  fp2_t zu2;
  const fp2_t den = sswu_den(u, &zu2);
  sswu_finish(xo, yo, u, zu2, den, fp2_inv(den), sqrt_m5);
}

// 3-isogeny E2' -> E2 (RFC 9380 E.3), output Jacobian without inversion.
BGV_NOINLINE g2_jac iso_map_g2(const fp2_t& x, const fp2_t& y) {
  const fp2_t xnum[4] = BGV_ISO_XNUM;
  const fp2_t xden[2] = BGV_ISO_XDEN;
  const fp2_t ynum[4] = BGV_ISO_YNUM;
  const fp2_t yden[3] = BGV_ISO_YDEN;
  fp2_t x2 = fp2_sqr(x);
  fp2_t x3 = fp2_mul(x2, x);
  fp2_t xn = fp2_add(fp2_add(fp2_mul(xnum[3], x3), fp2_mul(xnum[2], x2)), fp2_add(fp2_mul(xnum[1], x), xnum[0]));
  fp2_t xd = fp2_add(fp2_add(x2, fp2_mul(xden[1], x)), xden[0]);
  fp2_t yn = fp2_add(fp2_add(fp2_mul(ynum[3], x3), fp2_mul(ynum[2], x2)), fp2_add(fp2_mul(ynum[1], x), ynum[0]));
  fp2_t yd = fp2_add(fp2_add(x3, fp2_mul(yden[2], x2)), fp2_add(fp2_mul(yden[1], x), yden[0]));
  g2_jac r;
  r.z = fp2_mul(xd, yd);
  r.x = fp2_mul(fp2_mul(xn, yd), r.z);
  r.y = fp2_mul(fp2_mul(fp2_mul(y, yn), xd), fp2_sqr(r.z));
  return r;
}

// Simplified SWU on E2' straight to Jacobian coordinates, with no inversion (RFC 9380 6.6.2;
// x = X/Z^2, y = Y/Z^3).  x1 = x1n / x1d, so gx1 = U / V with V = x1d^3, and the square root
// of the ratio runs through the norm method of fp2_sqrt_or_z on U/V = w/n, w = U conj(V),
// n = N(V) in Fp: w/n is a square iff w is (n^2 is), sqrt(N(w/n)) = sqrt(N(w))/n, d = d'/n,
// and with T = n (d' n^3)^((p-3)/4)
//     d^((p+1)/4) = d' T,   h1 d^((p-3)/4) = h1' T,   d^((p-1)/2) = d' n T^2
// (n^(p-1) = 1), so the same two (p-3)/4 exponentiations as sqrt(g) give sqrt(U/V) and
// the inversion of the affine map is gone.  The same point as sswu_g2 (tests/test_hostsim_math.py).
template <class PW>
BGV_NOINLINE g2_jac sswu_g2_jac_t(const fp2_t& u, const fp_t& sqrt_m5) {
  const fp2_t Z = BGV_SSWU_Z, A = BGV_SSWU_A, B = BGV_SSWU_B;
  const fp2_t tv1 = fp2_mul(Z, fp2_sqr(u));
  const fp2_t tv2 = fp2_add(fp2_sqr(tv1), tv1);
  const bool exc = fp2_is_zero(tv2);  // x1 = B / (Z A)
  const fp2_t x1n = fp2_select(exc, fp2_neg(fp2_mul(B, fp2_add(tv2, fp2_one()))), B);
  const fp2_t x1d = fp2_select(exc, fp2_mul(A, tv2), fp2_mul(Z, A));
  const fp2_t d2 = fp2_sqr(x1d);
  const fp2_t V = fp2_mul(d2, x1d);
  const fp2_t U = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1n), fp2_mul(A, d2)), x1n), fp2_mul(B, V));
  const fp2_t w = fp2_mul(U, fp2_conj(V));
  const fp_t n = fp_add(fp_sqr(V.c0), fp_sqr(V.c1));
  const fp_t nw = fp_add(fp_sqr(w.c0), fp_sqr(w.c1));
  const fp_t e = PW::p34(nw);
  const fp_t ne = fp_mul(nw, e);
  const bool sq = fp_eq(fp_mul(ne, e), fp_one()) || fp_is_zero(nw);
  const fp2_t h = fp2_select(sq, fp2_mul(Z, w), w);
  const fp_t gam = fp_select(sq, fp_mul(sqrt_m5, fp_neg(ne)), ne);
  const fp_t d = fp_select(fp_is_zero(h.c1), fp_half(fp_add(h.c0, gam)), h.c0);
  const fp_t T = fp_mul(n, PW::p34(fp_mul(d, fp_mul(fp_sqr(n), n))));
  const fp_t y0 = fp_mul(d, T), y1 = fp_half(fp_mul(h.c1, T));
  const bool qr = fp_eq(fp_mul(fp_mul(d, n), fp_sqr(T)), fp_one());
  fp2_t r;  // sqrt(gx1), or sqrt(Z gx1) when gx1 is not a square
  r.c0 = fp_select(qr, y1, y0);
  r.c1 = fp_select(qr, fp_neg(y0), y1);
  // x = x1 or x2 = tv1 x1; y = r or tv1 u r (= Z u^3 sqrt(Z gx1))
  const fp2_t xn = fp2_mul(x1n, x1d);
  fp2_t y = fp2_select(sq, fp2_mul(fp2_mul(tv1, u), r), r);
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  g2_jac o;
  o.x = fp2_select(sq, fp2_mul(tv1, xn), xn);
  o.y = fp2_mul(y, V);
  o.z = x1d;
  return o;
}
BGV_HD g2_jac sswu_g2_jac(const fp2_t& u, const fp_t& sqrt_m5) { return sswu_g2_jac_t<bgv_pow_lane>(u, sqrt_m5); }

// 3-isogeny E2' -> E2 (RFC 9380 E.3) of a Jacobian point: the rational maps in x = X/Z^2
// homogenized with z2 = Z^2 (XN = xnum z2^3, XD = xden z2^2, YN = ynum z2^3, YD = yden z2^3),
// x' = XN / (XD z2), y' = Y YN / (Z^3 YD); output (A D W, C B W^2, W) with A/B = x',
// C/D = y', W = B D.
BGV_NOINLINE g2_jac iso_map_g2_jac(const g2_jac& p) {
  const fp2_t xnum[4] = BGV_ISO_XNUM;
  const fp2_t xden[2] = BGV_ISO_XDEN;
  const fp2_t ynum[4] = BGV_ISO_YNUM;
  const fp2_t yden[3] = BGV_ISO_YDEN;
  const fp2_t X = p.x, z2 = fp2_sqr(p.z);
  const fp2_t z4 = fp2_sqr(z2), z6 = fp2_mul(z4, z2);
  const fp2_t X2 = fp2_sqr(X), X3 = fp2_mul(X2, X);
  const fp2_t X2z2 = fp2_mul(X2, z2), Xz4 = fp2_mul(X, z4);
  const fp2_t XN = fp2_add(fp2_add(fp2_mul(xnum[3], X3), fp2_mul(xnum[2], X2z2)),
                           fp2_add(fp2_mul(xnum[1], Xz4), fp2_mul(xnum[0], z6)));
  const fp2_t XD = fp2_add(fp2_add(X2, fp2_mul(xden[1], fp2_mul(X, z2))), fp2_mul(xden[0], z4));
  const fp2_t YN = fp2_add(fp2_add(fp2_mul(ynum[3], X3), fp2_mul(ynum[2], X2z2)),
                           fp2_add(fp2_mul(ynum[1], Xz4), fp2_mul(ynum[0], z6)));
  const fp2_t YD = fp2_add(fp2_add(X3, fp2_mul(yden[2], X2z2)), fp2_add(fp2_mul(yden[1], Xz4), fp2_mul(yden[0], z6)));
  const fp2_t Bq = fp2_mul(XD, z2);
  const fp2_t Dq = fp2_mul(fp2_mul(p.z, z2), YD);
  const fp2_t Cq = fp2_mul(p.y, YN);
  g2_jac r;
  r.z = fp2_mul(Bq, Dq);
  r.x = fp2_mul(fp2_mul(XN, Dq), r.z);
  r.y = fp2_mul(fp2_mul(Cq, Bq), fp2_sqr(r.z));
  return r;
}

// Full hash_to_G2 of one message: a Jacobian point in G2 (both maps in Jacobian form, no
// inversion anywhere).
BGV_NOINLINE g2_jac hash_to_g2(const uint8_t* msg, uint32_t len) {
  fp2_t u0, u1;
  hash_to_field_fp2(&u0, &u1, msg, len);
  const fp_t sm5 = fp_sqrt_minus5();
  const g2_jac q0 = iso_map_g2_jac(sswu_g2_jac(u0, sm5));
  const g2_jac q1 = iso_map_g2_jac(sswu_g2_jac(u1, sm5));
  return g2_clear_cofactor(jac_add(q0, q1));
}
