// CPU restatement of Lodestar's BLS verify path — TEST INFRASTRUCTURE / CPU BASELINE ONLY.
//
// An independent C++ implementation (6 x 64-bit limbs, unsigned __int128
// Montgomery products, the x86 analogue of blst's mulx path) of what
// @chainsafe/blst@0.2.4 -> blst computes for
//   packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39   (batch vs single verify)
//   packages/beacon-node/src/chain/bls/multithread/worker.ts:32-108  (chunks of >= 16 jobs, per-job retry)
//   packages/beacon-node/src/chain/bls/multithread/index.ts:134-174,386-401 (128-set jobs, worker packages)
// with a BlsMultiThreadWorkerPool-style thread pool of nproc workers
// (multithread/poolSize.ts:7).  It shares no code with the HIP kernels
// (lodestar_amd/csrc); tests/test_cpu_oracle.py pins it to the golden vectors of
// the Python oracle.  Used by bench.py's cpu_baseline leg and by large-batch
// cross-checks; never by the product path.
//
// Build: oracle/cpu/Makefile -> oracle/cpu/libblscpu.so (g++ -O3 -march=native).
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <thread>
#include <vector>

typedef unsigned __int128 u128;

// ---------------------------------------------------------------------------
// Fp: 6 x 64-bit limbs, Montgomery R = 2^384
// ---------------------------------------------------------------------------
struct Fp {
  uint64_t l[6];
};
static const uint64_t PL[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                               0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static uint64_t N0;  // -p^-1 mod 2^64
static Fp ONE, R2;   // R mod p, R^2 mod p

static inline bool geq_p(const uint64_t a[6]) {
  for (int i = 5; i >= 0; --i) {
    if (a[i] > PL[i]) return true;
    if (a[i] < PL[i]) return false;
  }
  return true;
}
static inline void sub_p(uint64_t a[6]) {
  u128 b = 0;
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a[i] - PL[i] - (uint64_t)b;
    a[i] = (uint64_t)d;
    b = (d >> 64) & 1;
  }
}
static inline Fp fadd(const Fp& a, const Fp& b) {
  Fp r;
  u128 c = 0;
  for (int i = 0; i < 6; ++i) {
    c += (u128)a.l[i] + b.l[i];
    r.l[i] = (uint64_t)c;
    c >>= 64;
  }
  if (c || geq_p(r.l)) sub_p(r.l);
  return r;
}
static inline Fp fsub(const Fp& a, const Fp& b) {
  Fp r;
  u128 bo = 0;
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a.l[i] - b.l[i] - (uint64_t)bo;
    r.l[i] = (uint64_t)d;
    bo = (d >> 64) & 1;
  }
  if (bo) {
    u128 c = 0;
    for (int i = 0; i < 6; ++i) {
      c += (u128)r.l[i] + PL[i];
      r.l[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  return r;
}
static inline bool fzero(const Fp& a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3] | a.l[4] | a.l[5]) == 0; }
static inline bool feq(const Fp& a, const Fp& b) { return memcmp(a.l, b.l, 48) == 0; }
static inline Fp fneg(const Fp& a) { return fzero(a) ? a : fsub(Fp{{0, 0, 0, 0, 0, 0}}, a); }
static inline Fp fmul(const Fp& a, const Fp& b) {
  // CIOS, fully unrolled; the 7th/8th accumulator words carry the overflow
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0, t6 = 0;
#define MAC(t, x, y, c)                          \
  {                                              \
    u128 s_ = (u128)(x) * (y) + (t) + (c);       \
    t = (uint64_t)s_;                            \
    c = (uint64_t)(s_ >> 64);                    \
  }
#pragma GCC unroll 6
  for (int i = 0; i < 6; ++i) {
    const uint64_t ai = a.l[i];
    uint64_t c = 0;
    MAC(t0, ai, b.l[0], c) MAC(t1, ai, b.l[1], c) MAC(t2, ai, b.l[2], c)
    MAC(t3, ai, b.l[3], c) MAC(t4, ai, b.l[4], c) MAC(t5, ai, b.l[5], c)
    u128 s = (u128)t6 + c;
    t6 = (uint64_t)s;
    const uint64_t t7 = (uint64_t)(s >> 64);
    const uint64_t m = t0 * N0;
    c = 0;
    uint64_t dummy = t0;
    MAC(dummy, m, PL[0], c)
    MAC(t1, m, PL[1], c) MAC(t2, m, PL[2], c) MAC(t3, m, PL[3], c) MAC(t4, m, PL[4], c) MAC(t5, m, PL[5], c)
    s = (u128)t6 + c;
    t0 = t1; t1 = t2; t2 = t3; t3 = t4; t4 = t5;
    t5 = (uint64_t)s;
    t6 = t7 + (uint64_t)(s >> 64);
  }
#undef MAC
  Fp r = {{t0, t1, t2, t3, t4, t5}};
  if (t6 || geq_p(r.l)) sub_p(r.l);
  return r;
}
static inline Fp fsqr(const Fp& a) { return fmul(a, a); }
static Fp fpow(const Fp& a, const uint64_t* e, int nlimbs) {
  Fp r = ONE;
  for (int i = nlimbs * 64 - 1; i >= 0; --i) {
    r = fsqr(r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = fmul(r, a);
  }
  return r;
}
static uint64_t E_PM2[6], E_SQRT[6], E_LEG[6];  // p-2, (p+1)/4, (p-1)/2
static Fp finv(const Fp& a) { return fpow(a, E_PM2, 6); }
static Fp to_mont(const Fp& raw) { return fmul(raw, R2); }
static Fp from_mont(const Fp& a) { return fmul(a, Fp{{1, 0, 0, 0, 0, 0}}); }
static Fp fp_from_be(const uint8_t* b) {
  Fp r;
  for (int i = 0; i < 6; ++i) {
    uint64_t v = 0;
    for (int k = 0; k < 8; ++k) v = (v << 8) | b[(5 - i) * 8 + k];
    r.l[i] = v;
  }
  return r;
}
static void fp_to_be(uint8_t* b, const Fp& raw) {
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 8; ++k) b[(5 - i) * 8 + k] = (uint8_t)(raw.l[i] >> (56 - 8 * k));
}
static bool raw_lt_p(const Fp& a) { return !geq_p(a.l); }
static Fp fsmall(uint64_t v) { return to_mont(Fp{{v, 0, 0, 0, 0, 0}}); }
static bool fsqrt(Fp* out, const Fp& a) {
  Fp s = fpow(a, E_SQRT, 6);
  *out = s;
  return feq(fsqr(s), a);
}
static bool lex_largest(const Fp& a) {  // raw(a) > (p-1)/2
  Fp r = from_mont(a);
  Fp h = {{E_LEG[0], E_LEG[1], E_LEG[2], E_LEG[3], E_LEG[4], E_LEG[5]}};
  for (int i = 5; i >= 0; --i) {
    if (r.l[i] > h.l[i]) return true;
    if (r.l[i] < h.l[i]) return false;
  }
  return false;
}

// ---------------------------------------------------------------------------
// Fp2 = Fp[i]/(i^2+1), Fp6 = Fp2[v]/(v^3-(1+i)), Fp12 = Fp6[w]/(w^2-v)
// ---------------------------------------------------------------------------
struct Fp2 {
  Fp a, b;
};
static inline Fp2 f2add(const Fp2& x, const Fp2& y) { return {fadd(x.a, y.a), fadd(x.b, y.b)}; }
static inline Fp2 f2sub(const Fp2& x, const Fp2& y) { return {fsub(x.a, y.a), fsub(x.b, y.b)}; }
static inline Fp2 f2neg(const Fp2& x) { return {fneg(x.a), fneg(x.b)}; }
static inline Fp2 f2conj(const Fp2& x) { return {x.a, fneg(x.b)}; }
static inline Fp2 f2mul(const Fp2& x, const Fp2& y) {
  Fp t0 = fmul(x.a, y.a), t1 = fmul(x.b, y.b);
  Fp t2 = fmul(fadd(x.a, x.b), fadd(y.a, y.b));
  return {fsub(t0, t1), fsub(fsub(t2, t0), t1)};
}
static inline Fp2 f2sqr(const Fp2& x) { return {fmul(fadd(x.a, x.b), fsub(x.a, x.b)), fadd(fmul(x.a, x.b), fmul(x.a, x.b))}; }
static inline Fp2 f2mulfp(const Fp2& x, const Fp& k) { return {fmul(x.a, k), fmul(x.b, k)}; }
static inline Fp2 f2xi(const Fp2& x) { return {fsub(x.a, x.b), fadd(x.a, x.b)}; }  // * (1 + i)
static inline bool f2zero(const Fp2& x) { return fzero(x.a) && fzero(x.b); }
static inline bool f2eq(const Fp2& x, const Fp2& y) { return feq(x.a, y.a) && feq(x.b, y.b); }
static Fp2 F2ONE, F2ZERO;
static Fp2 f2inv(const Fp2& x) {
  Fp n = finv(fadd(fsqr(x.a), fsqr(x.b)));
  return {fmul(x.a, n), fneg(fmul(x.b, n))};
}
static bool f2sqrt(Fp2* out, const Fp2& x) {
  // complex method: a1 == 0 special case, else norm root
  if (fzero(x.b)) {
    Fp s;
    if (fsqrt(&s, x.a)) {
      *out = {s, Fp{}};
      return true;
    }
    if (fsqrt(&s, fneg(x.a))) {
      *out = {Fp{}, s};
      return true;
    }
    return false;
  }
  Fp g;
  if (!fsqrt(&g, fadd(fsqr(x.a), fsqr(x.b)))) return false;
  static const Fp inv2 = finv(fsmall(2));
  Fp d = fmul(fadd(x.a, g), inv2), x0;
  if (!fsqrt(&x0, d)) {
    d = fmul(fsub(x.a, g), inv2);
    if (!fsqrt(&x0, d)) return false;
  }
  Fp x1 = fmul(x.b, finv(fadd(x0, x0)));
  *out = {x0, x1};
  return f2eq(f2sqr(*out), x);
}
static bool f2lex_largest(const Fp2& y) { return fzero(y.b) ? lex_largest(y.a) : lex_largest(y.b); }
static uint32_t f2sgn0(const Fp2& x) {
  Fp a0 = from_mont(x.a), a1 = from_mont(x.b);
  return (uint32_t)((a0.l[0] & 1) | (fzero(a0) & (a1.l[0] & 1)));
}

struct Fp6 {
  Fp2 c0, c1, c2;
};
struct Fp12 {
  Fp6 a, b;
};
static inline Fp6 f6add(const Fp6& x, const Fp6& y) { return {f2add(x.c0, y.c0), f2add(x.c1, y.c1), f2add(x.c2, y.c2)}; }
static inline Fp6 f6sub(const Fp6& x, const Fp6& y) { return {f2sub(x.c0, y.c0), f2sub(x.c1, y.c1), f2sub(x.c2, y.c2)}; }
static inline Fp6 f6neg(const Fp6& x) { return {f2neg(x.c0), f2neg(x.c1), f2neg(x.c2)}; }
static inline Fp6 f6v(const Fp6& x) { return {f2xi(x.c2), x.c0, x.c1}; }
static Fp6 f6mul(const Fp6& x, const Fp6& y) {
  Fp2 t0 = f2mul(x.c0, y.c0), t1 = f2mul(x.c1, y.c1), t2 = f2mul(x.c2, y.c2);
  Fp2 c0 = f2add(f2xi(f2sub(f2sub(f2mul(f2add(x.c1, x.c2), f2add(y.c1, y.c2)), t1), t2)), t0);
  Fp2 c1 = f2add(f2sub(f2sub(f2mul(f2add(x.c0, x.c1), f2add(y.c0, y.c1)), t0), t1), f2xi(t2));
  Fp2 c2 = f2add(f2sub(f2sub(f2mul(f2add(x.c0, x.c2), f2add(y.c0, y.c2)), t0), t2), t1);
  return {c0, c1, c2};
}
static Fp6 f6inv(const Fp6& x) {
  Fp2 t0 = f2sub(f2sqr(x.c0), f2xi(f2mul(x.c1, x.c2)));
  Fp2 t1 = f2sub(f2xi(f2sqr(x.c2)), f2mul(x.c0, x.c1));
  Fp2 t2 = f2sub(f2sqr(x.c1), f2mul(x.c0, x.c2));
  Fp2 dn = f2add(f2mul(x.c0, t0), f2xi(f2add(f2mul(x.c2, t1), f2mul(x.c1, t2))));
  Fp2 di = f2inv(dn);
  return {f2mul(t0, di), f2mul(t1, di), f2mul(t2, di)};
}
static Fp12 f12mul(const Fp12& x, const Fp12& y) {
  Fp6 t0 = f6mul(x.a, y.a), t1 = f6mul(x.b, y.b);
  Fp6 c1 = f6sub(f6sub(f6mul(f6add(x.a, x.b), f6add(y.a, y.b)), t0), t1);
  return {f6add(t0, f6v(t1)), c1};
}
static Fp12 f12sqr(const Fp12& x) {
  Fp6 t = f6mul(x.a, x.b);
  Fp6 s = f6mul(f6add(x.a, x.b), f6add(x.a, f6v(x.b)));
  return {f6sub(f6sub(s, t), f6v(t)), f6add(t, t)};
}
static Fp12 f12conj(const Fp12& x) { return {x.a, f6neg(x.b)}; }
static Fp12 f12inv(const Fp12& x) {
  Fp6 n = f6inv(f6sub(f6mul(x.a, x.a), f6v(f6mul(x.b, x.b))));
  return {f6mul(x.a, n), f6neg(f6mul(x.b, n))};
}
static Fp12 F12ONE;
static bool f12one(const Fp12& x) { return memcmp(&x, &F12ONE, sizeof(Fp12)) == 0; }
static Fp2 FROB[6];  // xi^(j(p-1)/6), flat w^j
static Fp12 f12frob(const Fp12& x) {
  // tower a.c0,a.c1,a.c2 = w^0,w^2,w^4; b.c0,b.c1,b.c2 = w^1,w^3,w^5
  return {{f2conj(x.a.c0), f2mul(f2conj(x.a.c1), FROB[2]), f2mul(f2conj(x.a.c2), FROB[4])},
          {f2mul(f2conj(x.b.c0), FROB[1]), f2mul(f2conj(x.b.c1), FROB[3]), f2mul(f2conj(x.b.c2), FROB[5])}};
}
// Granger-Scott cyclotomic squaring
static void fp4sq(Fp2* c0, Fp2* c1, const Fp2& a, const Fp2& b) {
  Fp2 t0 = f2sqr(a), t1 = f2sqr(b);
  *c0 = f2add(f2xi(t1), t0);
  *c1 = f2sub(f2sub(f2sqr(f2add(a, b)), t0), t1);
}
static Fp12 f12cyc(const Fp12& f) {
  Fp2 z0 = f.a.c0, z4 = f.a.c1, z3 = f.a.c2, z2 = f.b.c0, z1 = f.b.c1, z5 = f.b.c2, t0, t1, t2, t3;
  fp4sq(&t0, &t1, z0, z1);
  z0 = f2add(f2add(f2sub(t0, z0), f2sub(t0, z0)), t0);
  z1 = f2add(f2add(f2add(t1, z1), f2add(t1, z1)), t1);
  fp4sq(&t0, &t1, z2, z3);
  fp4sq(&t2, &t3, z4, z5);
  z4 = f2add(f2add(f2sub(t0, z4), f2sub(t0, z4)), t0);
  z5 = f2add(f2add(f2add(t1, z5), f2add(t1, z5)), t1);
  t0 = f2xi(t3);
  z2 = f2add(f2add(f2add(t0, z2), f2add(t0, z2)), t0);
  z3 = f2add(f2add(f2sub(t2, z3), f2sub(t2, z3)), t2);
  return {{z0, z4, z3}, {z2, z1, z5}};
}
static const uint64_t XABS = 0xd201000000010000ULL;
static Fp12 cyc_pow_x(const Fp12& a) {  // a^x, x < 0
  Fp12 r = a;
  for (int i = 62; i >= 0; --i) {
    r = f12cyc(r);
    if ((XABS >> i) & 1) r = f12mul(r, a);
  }
  return f12conj(r);
}
// f^((p^12-1)/r) == 1 ?  Hard part via 3(p^4-p^2+1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3.
static bool final_exp_is_one(const Fp12& f) {
  Fp12 t = f12mul(f12conj(f), f12inv(f));
  t = f12mul(f12frob(f12frob(t)), t);
  Fp12 a = f12mul(cyc_pow_x(t), f12conj(t));
  a = f12mul(cyc_pow_x(a), f12conj(a));
  a = f12mul(cyc_pow_x(a), f12frob(a));
  Fp12 b = cyc_pow_x(cyc_pow_x(a));
  b = f12mul(f12mul(b, f12frob(f12frob(a))), f12conj(a));
  return f12one(f12mul(b, f12mul(f12cyc(t), t)));
}

// ---------------------------------------------------------------------------
// Curves (Jacobian; a = 0).  E1: y^2 = x^3 + 4, E2: y^2 = x^3 + 4(1+i)
// ---------------------------------------------------------------------------
template <class F>
struct Jac {
  F x, y, z;
};
struct FOps1 {
  typedef Fp F;
  static F add(const F& a, const F& b) { return fadd(a, b); }
  static F sub(const F& a, const F& b) { return fsub(a, b); }
  static F mul(const F& a, const F& b) { return fmul(a, b); }
  static F sqr(const F& a) { return fsqr(a); }
  static F neg(const F& a) { return fneg(a); }
  static bool zero(const F& a) { return fzero(a); }
  static F inv(const F& a) { return finv(a); }
  static F one() { return ONE; }
};
struct FOps2 {
  typedef Fp2 F;
  static F add(const F& a, const F& b) { return f2add(a, b); }
  static F sub(const F& a, const F& b) { return f2sub(a, b); }
  static F mul(const F& a, const F& b) { return f2mul(a, b); }
  static F sqr(const F& a) { return f2sqr(a); }
  static F neg(const F& a) { return f2neg(a); }
  static bool zero(const F& a) { return f2zero(a); }
  static F inv(const F& a) { return f2inv(a); }
  static F one() { return F2ONE; }
};
template <class O>
static Jac<typename O::F> jinf() {
  return {O::one(), O::one(), typename O::F{}};
}
template <class O>
static Jac<typename O::F> jdbl(const Jac<typename O::F>& p) {
  typedef typename O::F F;
  if (O::zero(p.z)) return p;
  F A = O::sqr(p.x), B = O::sqr(p.y), C = O::sqr(B);
  F D = O::sub(O::sub(O::sqr(O::add(p.x, B)), A), C);
  D = O::add(D, D);
  F E = O::add(O::add(A, A), A), Ff = O::sqr(E);
  Jac<F> r;
  r.x = O::sub(Ff, O::add(D, D));
  F C8 = O::add(C, C);
  C8 = O::add(C8, C8);
  C8 = O::add(C8, C8);
  r.y = O::sub(O::mul(E, O::sub(D, r.x)), C8);
  r.z = O::mul(p.y, p.z);
  r.z = O::add(r.z, r.z);
  return r;
}
template <class O>
static Jac<typename O::F> jadd(const Jac<typename O::F>& p, const Jac<typename O::F>& q) {
  typedef typename O::F F;
  if (O::zero(p.z)) return q;
  if (O::zero(q.z)) return p;
  F z1z1 = O::sqr(p.z), z2z2 = O::sqr(q.z);
  F u1 = O::mul(p.x, z2z2), u2 = O::mul(q.x, z1z1);
  F s1 = O::mul(O::mul(p.y, q.z), z2z2), s2 = O::mul(O::mul(q.y, p.z), z1z1);
  F h = O::sub(u2, u1), rr = O::sub(s2, s1);
  if (O::zero(h)) {
    if (O::zero(rr)) return jdbl<O>(p);
    return jinf<O>();
  }
  rr = O::add(rr, rr);
  F i = O::sqr(O::add(h, h)), j = O::mul(h, i), v = O::mul(u1, i);
  Jac<F> r;
  r.x = O::sub(O::sub(O::sqr(rr), j), O::add(v, v));
  F s1j = O::mul(s1, j);
  r.y = O::sub(O::mul(rr, O::sub(v, r.x)), O::add(s1j, s1j));
  r.z = O::mul(O::sub(O::sub(O::sqr(O::add(p.z, q.z)), z1z1), z2z2), h);
  return r;
}
template <class O>
static Jac<typename O::F> jneg(const Jac<typename O::F>& p) {
  return {p.x, O::neg(p.y), p.z};
}
// [k]P, 4-bit fixed window over nbits
template <class O>
static Jac<typename O::F> jmul(const Jac<typename O::F>& p, const uint64_t* k, int nbits) {
  typedef typename O::F F;
  Jac<F> tab[16];
  tab[0] = jinf<O>();
  tab[1] = p;
  for (int i = 2; i < 16; ++i) tab[i] = jadd<O>(tab[i - 1], p);
  Jac<F> acc = jinf<O>();
  for (int i = ((nbits + 3) / 4) * 4 - 4; i >= 0; i -= 4) {
    for (int d = 0; d < 4; ++d) acc = jdbl<O>(acc);
    const unsigned w = (unsigned)((k[i >> 6] >> (i & 63)) & 15);
    if (w) acc = jadd<O>(acc, tab[w]);
  }
  return acc;
}
template <class O>
static bool jaff(typename O::F* x, typename O::F* y, const Jac<typename O::F>& p) {
  if (O::zero(p.z)) return false;
  typename O::F zi = O::inv(p.z), zi2 = O::sqr(zi);
  *x = O::mul(p.x, zi2);
  *y = O::mul(p.y, O::mul(zi2, zi));
  return true;
}
template <class O>
static bool jeq(const Jac<typename O::F>& p, const Jac<typename O::F>& q) {
  typedef typename O::F F;
  if (O::zero(p.z) || O::zero(q.z)) return O::zero(p.z) && O::zero(q.z);
  F z1z1 = O::sqr(p.z), z2z2 = O::sqr(q.z);
  F a = O::sub(O::mul(p.x, z2z2), O::mul(q.x, z1z1));
  F b = O::sub(O::mul(O::mul(p.y, q.z), z2z2), O::mul(O::mul(q.y, p.z), z1z1));
  return O::zero(a) && O::zero(b);
}
typedef Jac<Fp> G1;
typedef Jac<Fp2> G2;
static Fp2 PSI_CX, PSI_CY;
static G2 psi(const G2& p) { return {f2mul(f2conj(p.x), PSI_CX), f2mul(f2conj(p.y), PSI_CY), f2conj(p.z)}; }
static G2 g2_mul_x(const G2& p) {  // [x]P, x = -|x|
  G2 acc = p;
  for (int i = 62; i >= 0; --i) {
    acc = jdbl<FOps2>(acc);
    if ((XABS >> i) & 1) acc = jadd<FOps2>(acc, p);
  }
  return jneg<FOps2>(acc);
}
static bool g2_in_group(const G2& p) { return jeq<FOps2>(psi(p), g2_mul_x(p)); }
static Fp2 B2;
static Fp B1;
static Fp G1X, G1Y;

// 96-byte compressed signature -> affine G2; returns BLST code (0 ok), *inf for infinity
static int g2_uncompress(Fp2* x, Fp2* y, bool* inf, const uint8_t* b) {
  *inf = false;
  if (!(b[0] & 0x80)) return 1;
  if (b[0] & 0x40) {
    uint8_t acc = b[0] & 0x3f;
    for (int i = 1; i < 96; ++i) acc |= b[i];
    if (acc) return 1;
    *inf = true;
    return 0;
  }
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  Fp x1 = fp_from_be(t), x0 = fp_from_be(b + 48);
  if (!raw_lt_p(x1) || !raw_lt_p(x0)) return 1;
  *x = {to_mont(x0), to_mont(x1)};
  Fp2 yy;
  if (!f2sqrt(&yy, f2add(f2mul(f2sqr(*x), *x), B2))) return 2;
  if (f2lex_largest(yy) != ((b[0] & 0x20) != 0)) yy = f2neg(yy);
  *y = yy;
  return 0;
}

// ---------------------------------------------------------------------------
// hash_to_G2 (RFC 9380, BLS12381G2_XMD:SHA-256_SSWU_RO_, DST POP)
// ---------------------------------------------------------------------------
struct Sha256 {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len;
  size_t n;
  static uint32_t rotr(uint32_t x, int k) { return (x >> k) | (x << (32 - k)); }
  void init() {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(h, iv, 32);
    len = 0;
    n = 0;
  }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t k) {
    len += k;
    while (k) {
      size_t m = 64 - n < k ? 64 - n : k;
      memcpy(buf + n, p, m);
      n += m;
      p += m;
      k -= m;
      if (n == 64) {
        block(buf);
        n = 0;
      }
    }
  }
  void final(uint8_t out[32]) {
    uint64_t bits = len * 8;
    uint8_t pad = 0x80;
    update(&pad, 1);
    uint8_t z = 0;
    while (n != 56) update(&z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(lb, 8);
    for (int i = 0; i < 8; ++i)
      for (int k = 0; k < 4; ++k) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
  }
};
static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
static void expand_xmd(uint8_t* out, size_t len_out, const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen) {
  uint8_t b0[32], bi[32], z[64] = {0};
  const size_t ell = (len_out + 31) / 32;
  uint8_t lib[2] = {(uint8_t)(len_out >> 8), (uint8_t)len_out}, dl = (uint8_t)dlen, zero = 0;
  Sha256 s;
  s.init();
  s.update(z, 64);
  s.update(msg, mlen);
  s.update(lib, 2);
  s.update(&zero, 1);
  s.update(dst, dlen);
  s.update(&dl, 1);
  s.final(b0);
  uint8_t prev[32];
  memset(prev, 0, 32);
  for (size_t i = 1; i <= ell; ++i) {
    uint8_t x[32];
    for (int k = 0; k < 32; ++k) x[k] = (uint8_t)(b0[k] ^ (i > 1 ? prev[k] : 0));
    uint8_t ib = (uint8_t)i;
    s.init();
    s.update(i == 1 ? b0 : x, 32);
    s.update(&ib, 1);
    s.update(dst, dlen);
    s.update(&dl, 1);
    s.final(bi);
    memcpy(prev, bi, 32);
    size_t off = (i - 1) * 32, m = len_out - off < 32 ? len_out - off : 32;
    memcpy(out + off, bi, m);
  }
}
// 64 big-endian bytes mod p
static Fp fp_from_be64(const uint8_t* b) {
  // v = hi * 2^256 + lo with hi, lo 256-bit: mont(v) = mont(hi) * 2^256 + mont(lo)
  Fp hi = {{0, 0, 0, 0, 0, 0}}, lo = {{0, 0, 0, 0, 0, 0}};
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 8; ++k) {
      hi.l[i] = (hi.l[i] << 8) | b[(3 - i) * 8 + k];
      lo.l[i] = (lo.l[i] << 8) | b[32 + (3 - i) * 8 + k];
    }
  Fp two256 = to_mont(Fp{{0, 0, 0, 0, 1, 0}});
  return fadd(fmul(to_mont(hi), two256), to_mont(lo));
}
static Fp2 SSWU_A, SSWU_B, SSWU_Z, ISO_XN[4], ISO_XD[3], ISO_YN[4], ISO_YD[4];
static bool f2is_square(const Fp2& a) {
  Fp n = fadd(fsqr(a.a), fsqr(a.b));
  Fp l = fpow(n, E_LEG, 6);
  return fzero(n) || feq(l, ONE);
}
static void sswu(Fp2* xo, Fp2* yo, const Fp2& u) {
  Fp2 zu2 = f2mul(SSWU_Z, f2sqr(u));
  Fp2 den = f2add(f2sqr(zu2), zu2), x1;
  if (f2zero(den))
    x1 = f2mul(SSWU_B, f2inv(f2mul(SSWU_Z, SSWU_A)));
  else
    x1 = f2mul(f2mul(f2neg(SSWU_B), f2inv(SSWU_A)), f2add(F2ONE, f2inv(den)));
  Fp2 gx1 = f2add(f2mul(f2add(f2sqr(x1), SSWU_A), x1), SSWU_B), x, y;
  if (f2is_square(gx1)) {
    x = x1;
    f2sqrt(&y, gx1);
  } else {
    x = f2mul(zu2, x1);
    f2sqrt(&y, f2add(f2mul(f2add(f2sqr(x), SSWU_A), x), SSWU_B));
  }
  if (f2sgn0(u) != f2sgn0(y)) y = f2neg(y);
  *xo = x;
  *yo = y;
}
static Fp2 poly(const Fp2* c, int n, const Fp2& x) {
  Fp2 acc = c[n - 1];
  for (int i = n - 2; i >= 0; --i) acc = f2add(f2mul(acc, x), c[i]);
  return acc;
}
static G2 iso_map(const Fp2& x, const Fp2& y) {
  Fp2 xn = poly(ISO_XN, 4, x), xd = poly(ISO_XD, 3, x), yn = poly(ISO_YN, 4, x), yd = poly(ISO_YD, 4, x);
  return {f2mul(xn, f2inv(xd)), f2mul(y, f2mul(yn, f2inv(yd))), F2ONE};
}
static G2 clear_cofactor(const G2& p) {
  G2 t1 = g2_mul_x(p), t2 = psi(p);
  G2 t3 = psi(psi(jdbl<FOps2>(p)));
  t3 = jadd<FOps2>(t3, jneg<FOps2>(t2));
  t2 = g2_mul_x(jadd<FOps2>(t1, t2));
  t3 = jadd<FOps2>(t3, t2);
  t3 = jadd<FOps2>(t3, jneg<FOps2>(t1));
  return jadd<FOps2>(t3, jneg<FOps2>(p));
}
static G2 hash_to_g2(const uint8_t* msg, size_t len) {
  uint8_t u[256];
  expand_xmd(u, 256, msg, len, (const uint8_t*)DST, sizeof(DST) - 1);
  Fp2 u0 = {fp_from_be64(u), fp_from_be64(u + 64)}, u1 = {fp_from_be64(u + 128), fp_from_be64(u + 192)};
  Fp2 x, y;
  sswu(&x, &y, u0);
  G2 q0 = iso_map(x, y);
  sswu(&x, &y, u1);
  G2 q1 = iso_map(x, y);
  return clear_cofactor(jadd<FOps2>(q0, q1));
}

// ---------------------------------------------------------------------------
// Miller loop (affine Q, Jacobian T, lines scaled into sparse w^0 / w^2 / w^3 slots)
// ---------------------------------------------------------------------------
static Fp12 mul_line(const Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3) {
  Fp12 line = {{l0, l2, F2ZERO}, {F2ZERO, l3, F2ZERO}};
  return f12mul(f, line);
}
static Fp12 miller(const Fp& px, const Fp& py, const Fp2& qx, const Fp2& qy) {
  G2 t = {qx, qy, F2ONE};
  Fp12 f = F12ONE;
  const Fp npx = fneg(px);
  for (int i = 62; i >= 0; --i) {
    if (i != 62) f = f12sqr(f);
    // doubling step with tangent line
    Fp2 A = f2sqr(t.x), B = f2sqr(t.y), C = f2sqr(B), ZZ = f2sqr(t.z);
    Fp2 D = f2sub(f2sub(f2sqr(f2add(t.x, B)), A), C);
    D = f2add(D, D);
    Fp2 E = f2add(f2add(A, A), A), F = f2sqr(E);
    Fp2 l0 = f2sub(f2mul(E, t.x), f2add(B, B));
    Fp2 l2 = f2mulfp(f2mul(E, ZZ), npx);
    Fp2 X3 = f2sub(F, f2add(D, D));
    Fp2 C8 = f2add(C, C);
    C8 = f2add(C8, C8);
    C8 = f2add(C8, C8);
    Fp2 Y3 = f2sub(f2mul(E, f2sub(D, X3)), C8);
    Fp2 Z3 = f2sub(f2sub(f2sqr(f2add(t.y, t.z)), B), ZZ);
    Fp2 l3 = f2mulfp(f2mul(Z3, ZZ), py);
    t = {X3, Y3, Z3};
    f = mul_line(f, l0, l2, l3);
    if ((XABS >> i) & 1) {
      Fp2 ZZ2 = f2sqr(t.z), U2 = f2mul(qx, ZZ2), S2 = f2mul(qy, f2mul(t.z, ZZ2));
      Fp2 H = f2sub(U2, t.x), HH = f2sqr(H), I = f2add(HH, HH);
      I = f2add(I, I);
      Fp2 J = f2mul(H, I), r = f2sub(S2, t.y);
      r = f2add(r, r);
      Fp2 V = f2mul(t.x, I);
      Fp2 X = f2sub(f2sub(f2sqr(r), J), f2add(V, V));
      Fp2 yj = f2mul(t.y, J);
      Fp2 Y = f2sub(f2mul(r, f2sub(V, X)), f2add(yj, yj));
      Fp2 Z = f2sub(f2sub(f2sqr(f2add(t.z, H)), ZZ2), HH);
      f = mul_line(f, f2sub(f2mul(r, qx), f2mul(qy, Z)), f2mulfp(r, npx), f2mulfp(Z, py));
      t = {X, Y, Z};
    }
  }
  return f12conj(f);
}

// ---------------------------------------------------------------------------
// Verify semantics
// ---------------------------------------------------------------------------
struct Set {
  Fp pkx, pky;  // affine pubkey (Montgomery), trusted
  bool pk_inf;
  const uint8_t* msg;
  const uint8_t* sig;
  uint32_t sig_len;
};
// returns 1 valid, 0 invalid, -code error (maybeBatch.ts:16-39 with blst semantics)
static int verify_maybe_batch(const Set* sets, size_t n, uint64_t* rng) {
  if (n == 0) return -21;
  std::vector<Fp2> sx(n), sy(n);
  std::vector<char> sinf(n);
  for (size_t i = 0; i < n; ++i) {  // Signature.fromBytes(sig, affine, validate=true)
    if (sets[i].sig_len != 96) return -8;
    bool inf;
    int rc = g2_uncompress(&sx[i], &sy[i], &inf, sets[i].sig);
    if (rc) return -rc;
    sinf[i] = inf;
    if (!inf && !g2_in_group(G2{sx[i], sy[i], F2ONE})) return -3;
  }
  if (n == 1) {  // core verify: e(pk, H(m)) * e(-G1, sig) == 1
    if (sets[0].pk_inf) return 0;
    Fp2 hx, hy;
    jaff<FOps2>(&hx, &hy, hash_to_g2(sets[0].msg, 32));
    Fp12 f = miller(sets[0].pkx, sets[0].pky, hx, hy);
    if (!sinf[0]) f = f12mul(f, miller(G1X, fneg(G1Y), sx[0], sy[0]));
    return final_exp_is_one(f) ? 1 : 0;
  }
  Fp12 f = F12ONE;
  G2 s = jinf<FOps2>();
  for (size_t i = 0; i < n; ++i) {
    uint64_t r;
    do {  // xorshift64* stream seeded per worker; nonzero 64-bit randomizers
      *rng ^= *rng >> 12;
      *rng ^= *rng << 25;
      *rng ^= *rng >> 27;
      r = *rng * 0x2545F4914F6CDD1DULL;
    } while (r == 0);
    if (!sinf[i]) s = jadd<FOps2>(s, jmul<FOps2>(G2{sx[i], sy[i], F2ONE}, &r, 64));
    if (sets[i].pk_inf) return -6;
    Fp px, py;
    jaff<FOps1>(&px, &py, jmul<FOps1>(G1{sets[i].pkx, sets[i].pky, ONE}, &r, 64));
    Fp2 hx, hy;
    jaff<FOps2>(&hx, &hy, hash_to_g2(sets[i].msg, 32));
    f = f12mul(f, miller(px, py, hx, hy));
  }
  Fp2 ax, ay;
  if (jaff<FOps2>(&ax, &ay, s)) f = f12mul(f, miller(G1X, fneg(G1Y), ax, ay));
  return final_exp_is_one(f) ? 1 : 0;
}

static void init_constants() {
  static bool done = false;
  if (done) return;
  // N0 = -p^-1 mod 2^64 (Newton)
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - PL[0] * inv;
  N0 = (uint64_t)0 - inv;
  // R mod p and R^2 mod p by doubling 1
  Fp x = {{1, 0, 0, 0, 0, 0}};
  auto dbl_raw = [](Fp v) {
    Fp r;
    uint64_t c = 0;
    for (int i = 0; i < 6; ++i) {
      uint64_t nv = (v.l[i] << 1) | c;
      c = v.l[i] >> 63;
      r.l[i] = nv;
    }
    if (c || geq_p(r.l)) sub_p(r.l);
    return r;
  };
  for (int i = 0; i < 384; ++i) x = dbl_raw(x);
  ONE = x;
  for (int i = 0; i < 384; ++i) x = dbl_raw(x);
  R2 = x;
  // exponents
  auto sub_small = [](uint64_t* o, uint64_t k) {
    memcpy(o, PL, 48);
    u128 b = k;
    for (int i = 0; i < 6 && b; ++i) {
      u128 d = (u128)o[i] - (uint64_t)b;
      o[i] = (uint64_t)d;
      b = (d >> 64) & 1;
    }
  };
  sub_small(E_PM2, 2);
  // (p+1)/4 and (p-1)/2
  uint64_t t[6];
  memcpy(t, PL, 48);
  u128 c = 1;
  for (int i = 0; i < 6; ++i) {
    c += t[i];
    t[i] = (uint64_t)c;
    c >>= 64;
  }
  for (int i = 0; i < 6; ++i) E_SQRT[i] = (t[i] >> 2) | (i < 5 ? t[i + 1] << 62 : 0);
  sub_small(t, 1);
  for (int i = 0; i < 6; ++i) E_LEG[i] = (t[i] >> 1) | (i < 5 ? t[i + 1] << 63 : 0);
  F2ONE = {ONE, Fp{}};
  F2ZERO = {Fp{}, Fp{}};
  F12ONE = {{F2ONE, F2ZERO, F2ZERO}, {F2ZERO, F2ZERO, F2ZERO}};
  B1 = fsmall(4);
  B2 = {fsmall(4), fsmall(4)};
  static const uint8_t g1x[48] = {0x17, 0xf1, 0xd3, 0xa7, 0x31, 0x97, 0xd7, 0x94, 0x26, 0x95, 0x63, 0x8c,
                                  0x4f, 0xa9, 0xac, 0x0f, 0xc3, 0x68, 0x8c, 0x4f, 0x97, 0x74, 0xb9, 0x05,
                                  0xa1, 0x4e, 0x3a, 0x3f, 0x17, 0x1b, 0xac, 0x58, 0x6c, 0x55, 0xe8, 0x3f,
                                  0xf9, 0x7a, 0x1a, 0xef, 0xfb, 0x3a, 0xf0, 0x0a, 0xdb, 0x22, 0xc6, 0xbb};
  static const uint8_t g1y[48] = {0x08, 0xb3, 0xf4, 0x81, 0xe3, 0xaa, 0xa0, 0xf1, 0xa0, 0x9e, 0x30, 0xed,
                                  0x74, 0x1d, 0x8a, 0xe4, 0xfc, 0xf5, 0xe0, 0x95, 0xd5, 0xd0, 0x0a, 0xf6,
                                  0x00, 0xdb, 0x18, 0xcb, 0x2c, 0x04, 0xb3, 0xed, 0xd0, 0x3c, 0xc7, 0x44,
                                  0xa2, 0x88, 0x8a, 0xe4, 0x0c, 0xaa, 0x23, 0x29, 0x46, 0xc5, 0xe7, 0xe1};
  G1X = to_mont(fp_from_be(g1x));
  G1Y = to_mont(fp_from_be(g1y));
  done = true;
}

// small-constant setup that needs field exponentiation (psi, Frobenius, SSWU, iso)
static Fp2 f2pow(Fp2 a, const uint64_t* e, int nl) {
  Fp2 r = F2ONE;
  for (int i = nl * 64 - 1; i >= 0; --i) {
    r = f2sqr(r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = f2mul(r, a);
  }
  return r;
}

extern "C" {

// Constants that the host passes in (raw big-endian, generated from oracle/bls12381.py
// by oracle/cpu/blscpu.py at load time): SSWU A/B/Z, iso coefficients.
static bool consts_ok = false;
int blscpu_init(const uint8_t* sswu_abz /*3 x 96*/, const uint8_t* iso /*(4+3+4+4) x 96*/) {
  init_constants();
  auto rd2 = [](const uint8_t* b) { return Fp2{to_mont(fp_from_be(b)), to_mont(fp_from_be(b + 48))}; };
  SSWU_A = rd2(sswu_abz);
  SSWU_B = rd2(sswu_abz + 96);
  SSWU_Z = rd2(sswu_abz + 192);
  const uint8_t* q = iso;
  for (int i = 0; i < 4; ++i, q += 96) ISO_XN[i] = rd2(q);
  for (int i = 0; i < 3; ++i, q += 96) ISO_XD[i] = rd2(q);
  for (int i = 0; i < 4; ++i, q += 96) ISO_YN[i] = rd2(q);
  for (int i = 0; i < 4; ++i, q += 96) ISO_YD[i] = rd2(q);
  // psi and Frobenius constants: xi^((p-1)/k)
  uint64_t e[6];
  Fp2 xi = {ONE, ONE};
  auto pm1_div = [&](uint64_t k) {  // (p-1)/k for k | p-1 (k in {2,3,6})
    uint64_t t[6];
    memcpy(t, PL, 48);
    t[0] -= 1;
    u128 rem = 0;
    for (int i = 5; i >= 0; --i) {
      u128 cur = (rem << 64) | t[i];
      e[i] = (uint64_t)(cur / k);
      rem = cur % k;
    }
  };
  pm1_div(6);
  Fp2 g1 = f2pow(xi, e, 6);
  FROB[0] = F2ONE;
  for (int j = 1; j < 6; ++j) FROB[j] = f2mul(FROB[j - 1], g1);
  pm1_div(3);
  PSI_CX = f2inv(f2pow(xi, e, 6));
  pm1_div(2);
  PSI_CY = f2inv(f2pow(xi, e, 6));
  consts_ok = true;
  return 0;
}

// hash_to_G2 -> 192-byte uncompressed (x.c1 | x.c0 | y.c1 | y.c0)
int blscpu_hash_to_g2(const uint8_t* msg, uint32_t len, uint8_t* out192) {
  if (!consts_ok) return -1;
  Fp2 x, y;
  if (!jaff<FOps2>(&x, &y, hash_to_g2(msg, len))) return 0;
  fp_to_be(out192, from_mont(x.b));
  fp_to_be(out192 + 48, from_mont(x.a));
  fp_to_be(out192 + 96, from_mont(y.b));
  fp_to_be(out192 + 144, from_mont(y.a));
  return 1;
}

// Verify njobs jobs the way BlsMultiThreadWorkerPool does:
//   pubkeys: per set an affine 96-byte uncompressed (x|y) record (already aggregated),
//   jobs:    [first_set, n_sets, batchable] triples;
//   mode 0:  worker semantics (batchable jobs in chunks of >= 16 jobs, retry per job),
//   mode 1:  every job alone.
// Work is split over `threads` workers in packages of ~128 sets (index.ts:386-401).
int blscpu_verify(const uint8_t* pk96, const uint8_t* msgs32, const uint8_t* sigs96, const uint32_t* sig_lens,
                  const uint32_t* jobs3, size_t njobs, int mode, int threads, uint64_t seed, int32_t* out) {
  if (!consts_ok) return -1;
  // packages of >= 128 sets of consecutive jobs
  std::vector<std::pair<size_t, size_t>> pkgs;
  for (size_t j = 0; j < njobs;) {
    size_t k = j, sets = 0;
    while (k < njobs && sets < 128) sets += jobs3[3 * k + 1], ++k;
    pkgs.push_back({j, k});
    j = k;
  }
  std::atomic<size_t> next(0);
  auto worker = [&](int wid) {
    uint64_t rng = seed ^ (0x9E3779B97F4A7C15ULL * (uint64_t)(wid + 1));
    if (!rng) rng = 1;
    for (;;) {
      size_t p = next.fetch_add(1);
      if (p >= pkgs.size()) return;
      auto mk = [&](size_t j, std::vector<Set>& v) {
        for (uint32_t q = 0; q < jobs3[3 * j + 1]; ++q) {
          size_t s = jobs3[3 * j] + q;
          Set st;
          const uint8_t* pk = pk96 + 96 * s;
          st.pk_inf = (pk[0] & 0x40) != 0;
          if (!st.pk_inf) {
            st.pkx = to_mont(fp_from_be(pk));
            st.pky = to_mont(fp_from_be(pk + 48));
          }
          st.msg = msgs32 + 32 * s;
          st.sig = sigs96 + 96 * s;
          st.sig_len = sig_lens[s];
          v.push_back(st);
        }
      };
      std::vector<size_t> batchable, alone;
      for (size_t j = pkgs[p].first; j < pkgs[p].second; ++j) {
        if (mode == 0 && jobs3[3 * j + 2])
          batchable.push_back(j);
        else
          alone.push_back(j);
      }
      // chunkifyMaximizeChunkSize(batchable, 16) (worker.ts:56)
      size_t cc = batchable.size() / 16;
      size_t per = cc <= 1 ? batchable.size() : (batchable.size() + cc - 1) / cc;
      for (size_t c0 = 0; c0 < batchable.size(); c0 += per) {
        std::vector<Set> all;
        size_t c1 = std::min(batchable.size(), c0 + per);
        for (size_t q = c0; q < c1; ++q) mk(batchable[q], all);
        int r = verify_maybe_batch(all.data(), all.size(), &rng);
        if (r == 1) {
          for (size_t q = c0; q < c1; ++q) out[batchable[q]] = 1;
        } else {
          for (size_t q = c0; q < c1; ++q) alone.push_back(batchable[q]);
        }
      }
      for (size_t j : alone) {
        std::vector<Set> v;
        mk(j, v);
        out[j] = verify_maybe_batch(v.data(), v.size(), &rng);
      }
    }
  };
  if (threads < 1) threads = 1;
  std::vector<std::thread> ts;
  for (int t = 1; t < threads; ++t) ts.emplace_back(worker, t);
  worker(0);
  for (auto& t : ts) t.join();
  return 0;
}
}

extern "C" {
// sk (32-byte big-endian) -> 96-byte uncompressed pubkey x|y (test data for the CPU baseline)
int blscpu_sk_to_pk96(const uint8_t* sk32, size_t n, uint8_t* out96) {
  if (!consts_ok) return -1;
  for (size_t i = 0; i < n; ++i) {
    uint64_t k[4];
    for (int w = 0; w < 4; ++w) {
      uint64_t v = 0;
      for (int b = 0; b < 8; ++b) v = (v << 8) | sk32[32 * i + (3 - w) * 8 + b];
      k[w] = v;
    }
    Fp x, y;
    if (!jaff<FOps1>(&x, &y, jmul<FOps1>(G1{G1X, G1Y, ONE}, k, 256))) {
      memset(out96 + 96 * i, 0, 96);
      out96[96 * i] = 0x40;
      continue;
    }
    fp_to_be(out96 + 96 * i, from_mont(x));
    fp_to_be(out96 + 96 * i + 48, from_mont(y));
  }
  return 0;
}
}
