"""Residue-number-system (RNS) Montgomery arithmetic for the latency path's Fp12 chains: the
constants (-> lodestar_amd/csrc/bgv_rns_consts.h) and an exact lane-level model of the device
algorithm (bgv_rns.h), checked here against big-integer arithmetic mod p and the oracle's
Fp12 operations.

    python tools/gen_rns.py            # self-check, then write the header
    python tools/gen_rns.py --check    # self-check only

Representation.  An Fp element is kept as the residues of an integer X (X = x M mod p, up to
a small multiple of p: X < 16 p) modulo 30 pseudo-Mersenne primes m = 2^28 - c, c < 2^10:
base B (15 moduli, product M ~ 2^420) and base B' (15 moduli, product M').  One lane holds one
residue, so an Fp value is 30 lanes and an Fp12 value 12 x 30 lanes (two coefficients per
wave, six waves).  Sums and products are lane-local; a Montgomery product of the integers
(Bajard / Kawamura RNS Montgomery: q = -s p^-1 mod M in B, extended to B' (fast, q^ = q +
alpha M), r = (s + q^ p) / M in B', extended back to B exactly) costs two base extensions,
each a 15-term dot product per lane over the other base's residues.  An Fp12 product sums
all 12 double-width Fp terms of a coefficient lane-locally and reduces once.

Bounds (checked by the model): operands X < 16 p; a coefficient's 12 products are < 16p * 32p
each, s < 6144 p^2 < M p; r = (s + q^ p) / M < s / M + 15 p < 16 p (alpha <= 14).  The second
extension's alpha is exact (Kawamura): sum_j xi_j / m_j = beta + r / M' with r / M' < 2^-34,
evaluated as sum_j xi_j floor(2^59 / m_j) / 2^59 (error < 2^-27) plus 2^-24, then floored.

Reference: the final exponentiation the latency path closes a call with (blst
verifyMultipleAggregateSignatures, chain/bls/maybeBatch.ts:18-25), bls_team.h tm_final_exp_u.
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
LB = 28           # bits of the 28-bit-limb Montgomery domain of the rest of the library
R28 = 1 << (LB * 14)  # its Montgomery constant 2^392
NB = 15           # moduli per base
MB = 28           # modulus bits
KNEG = 16         # negation constant K p (operand bound)
BETA_SHIFT = 59   # G_j = floor(2^59 / m_j)
BETA_ROUND = 1 << 35  # 2^-24 in the 2^59 fixed point


def is_prime(n):
    if n < 2:
        return False
    for q in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % q == 0:
            return n == q
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def pick_moduli():
    out, c = [], 1
    while len(out) < 2 * NB:
        if is_prime((1 << MB) - c):
            out.append((1 << MB) - c)
        c += 2
    assert (1 << MB) - out[-1] < (1 << 10)
    return out[:NB], out[NB:]


BASE, BASEP = pick_moduli()
MODS = BASE + BASEP
M = 1
for m in BASE:
    M *= m
MP = 1
for m in BASEP:
    MP *= m
assert M > 6144 * P and MP > 32 * P * (1 << 34)


# ------------------------------------------------------------------------------------------
# per-lane constants
# ------------------------------------------------------------------------------------------
def lane_consts():
    """Per lane i (0..29) a dict; the device keeps these in registers (bgv_rns_consts.h)."""
    out = []
    for i, m in enumerate(MODS):
        d = {"m": m, "c": (1 << MB) - m, "c16": 16 * ((1 << MB) - m)}
        d["kp"] = KNEG * P % m
        d["pm"] = P % m
        if i < NB:
            Mi = M // m
            d["xi"] = (-pow(P, -1, m) * pow(Mi, -1, m)) % m          # q_i M_i^-1 folded: xi = s C
            d["row"] = [(MP // mj) % m for mj in BASEP]               # BE2: |M'_j|_{m_i}
            d["mpc"] = (m - MP % m) % m                               # beta correction: -M' mod m_i
        else:
            j = i - NB
            Mj = MP // m
            d["row"] = [(M // mk) % m for mk in BASE]                 # BE1: |M_k|_{m'_j}
            d["minv"] = pow(M, -1, m)                                 # r = (s + q p) M^-1
            d["xi"] = pow(Mj, -1, m)                                  # xi'_j = r_j M'_j^-1
        d["l28"] = [pow(2, LB * k, m) for k in range(15)]             # 28-bit limbs -> residue
        out.append(d)
    return out


LANES = lane_consts()
GBETA = [(1 << BETA_SHIFT) // m for m in BASEP]
assert all(g < (1 << 32) for g in GBETA)


# ------------------------------------------------------------------------------------------
# the device's lane arithmetic
# ------------------------------------------------------------------------------------------
def red64(x, L):
    """x < 2^64 -> x mod m (bgv_rns.h rns_red): 2^32 = 16 c mod m, then 2^28 = c."""
    assert 0 <= x < (1 << 64)
    c16, c, m = L["c16"], L["c"], L["m"]
    y = (x >> 32) * c16 + (x & 0xFFFFFFFF)
    assert y < (1 << 64)
    z = (y >> 32) * c16 + (y & 0xFFFFFFFF)
    assert z < (1 << 34)
    w = (z >> MB) * c + (z & ((1 << MB) - 1))
    assert w < 2 * m
    return w - m if w >= m else w


def to_rns(X):
    return [X % m for m in MODS]


def from_rns_b(r):
    """CRT over base B (the integer the B lanes hold)."""
    x = 0
    for i, m in enumerate(BASE):
        Mi = M // m
        x += r[i] * Mi * pow(Mi, -1, m)
    return x % M


def from_rns_bp(r):
    x = 0
    for j, m in enumerate(BASEP):
        Mj = MP // m
        x += r[NB + j] * Mj * pow(Mj, -1, m)
    return x % MP


def mont_reduce(s):
    """s: 30 residues of a sum of products (each < 2^64 before the lane reduction, already
    reduced mod m here) -> r = s M^-1 mod p, 30 residues, exactly as the lanes compute it."""
    xi = [red64(s[i] * LANES[i]["xi"], LANES[i]) for i in range(NB)]
    r = [0] * 30
    xip = [0] * NB
    for j in range(NB):
        L = LANES[NB + j]
        acc = sum(xi[k] * L["row"][k] for k in range(NB))
        assert acc < (1 << 64)
        q = red64(acc, L)
        t = red64(s[NB + j] + q * L["pm"], L)
        r[NB + j] = red64(t * L["minv"], L)
        xip[j] = red64(r[NB + j] * L["xi"], L)
    bacc = sum(xip[j] * GBETA[j] for j in range(NB))
    assert bacc + BETA_ROUND < (1 << 64)
    beta = (bacc + BETA_ROUND) >> BETA_SHIFT
    for i in range(NB):
        L = LANES[i]
        acc = sum(xip[j] * L["row"][j] for j in range(NB)) + beta * L["mpc"]
        assert acc < (1 << 64)
        r[i] = red64(acc, L)
    return r, beta


def rns_int(r):
    xb, xbp = from_rns_b(r), from_rns_bp(r)
    assert xb == xbp, "bases disagree"
    return xb


def mont_mul(a, b):
    s = [red64(a[i] * b[i], LANES[i]) for i in range(30)]
    return mont_reduce(s)[0]


# Fp12 in the w-basis (oracle order: 6 Fp2 coefficients of w^k); the lane coefficient index
# c = 2k + e (e: 0 real, 1 imaginary part), as bls_team.h
def f12_terms(k, e):
    """the 6 (i, j, wrap) terms of output coefficient (k, e) of a product"""
    out = []
    for i in range(6):
        wrap = i > k
        j = k + 6 - i if wrap else k - i
        out.append((i, j, wrap))
    return out


def lane_mul12(A, B, c, i):
    """lane (c, i): the unreduced residue sum of output coefficient c of A * B (A, B: 12 x 30
    residues); the same 12 products as bls_team.h tm_mul_lane, negations as K p - x"""
    L = LANES[i]
    m, kp = L["m"], L["kp"]
    k, e = c >> 1, c & 1
    acc = 0
    for (ii, j, wrap) in f12_terms(k, e):
        x0, x1 = A[2 * ii][i], A[2 * ii + 1][i]
        y0, y1 = B[2 * j][i], B[2 * j + 1][i]
        d = y0 + (kp + m - y1)       # y0 - y1 + K p   (< 3m)
        s = y0 + y1                  # (< 2m)
        x1n = kp + m - x1            # K p - x1        (< 2m)
        X2 = x1 if e else x1n
        if wrap:
            Y1, Y2 = (s, d) if e else (d, s)
        else:
            Y1, Y2 = (y1, y0) if e else (y0, y1)
        acc += x0 * Y1 + X2 * Y2
    assert acc < (1 << 64)
    return red64(acc, L)


def rns12_mul(A, B):
    S = [[lane_mul12(A, B, c, i) for i in range(30)] for c in range(12)]
    return [mont_reduce(S[c])[0] for c in range(12)]


def f12_to_rns(f, scale=M):
    """oracle Fp12 (6 Fp2 in the w-basis) -> 12 x 30 residues of x * scale mod p"""
    out = []
    for k in range(6):
        for e in range(2):
            out.append(to_rns(f[k][e] * scale % P))
    return out


def rns_to_f12(A):
    """12 x 30 residues (M-form) -> oracle Fp12"""
    Minv = pow(M, -1, P)
    v = [rns_int(a) * Minv % P for a in A]
    return tuple((v[2 * k], v[2 * k + 1]) for k in range(6))


def check(n=40, seed=1):
    from oracle import bls12381 as o
    rnd = random.Random(seed)
    worst = 0
    for _ in range(n):
        x, y = rnd.randrange(KNEG * P), rnd.randrange(KNEG * P)
        r, beta = mont_reduce([red64(a * b, LANES[i]) for i, (a, b) in enumerate(zip(to_rns(x), to_rns(y)))])
        v = rns_int(r)
        assert v % P == x * y * pow(M, -1, P) % P
        assert v < KNEG * P
        worst = max(worst, v / P)
    # extremes: the largest operands
    for x in (0, 1, P - 1, KNEG * P - 1):
        for y in (0, KNEG * P - 1):
            v = rns_int(mont_mul(to_rns(x), to_rns(y)))
            assert v % P == x * y * pow(M, -1, P) % P and v < KNEG * P
    # Fp12 products against the oracle
    for _ in range(3):
        fa = tuple((rnd.randrange(P), rnd.randrange(P)) for _ in range(6))
        fb = tuple((rnd.randrange(P), rnd.randrange(P)) for _ in range(6))
        got = rns_to_f12(rns12_mul(f12_to_rns(fa), f12_to_rns(fb)))
        assert got == o.f12_mul(fa, fb)
        # chained: the outputs (< 16 p, unnormalized) as operands again
        A = rns12_mul(f12_to_rns(fa), f12_to_rns(fb))
        got2 = rns_to_f12(rns12_mul(A, A))
        assert got2 == o.f12_sqr(o.f12_mul(fa, fb))
        for a in A:
            assert rns_int(a) < KNEG * P
    return worst


def c_array(name, vals, ctype="uint32_t"):
    return "BGV_RNS_CONST %s %s[%d] = {%s};\n" % (ctype, name, len(vals), ", ".join("0x%xu" % v for v in vals))


def frob_consts():
    """w-basis Frobenius constants in RNS M-form: gamma_k = xi^(k (p - 1) / 6) (Fp2, for x -> x^p)
    and gamma2_k = xi^(k (p^2 - 1) / 6) (in Fp, for x -> x^(p^2)); oracle f12_frob's order"""
    from oracle import bls12381 as o
    g1, g2 = [], []
    for k in range(6):
        g = o.f2_pow(o.XI, k * (P - 1) // 6)
        h = o.f2_pow(o.XI, k * (P * P - 1) // 6)
        assert h[1] == 0
        g1.extend(to_rns(g[0] * M % P) + to_rns(g[1] * M % P))
        g2.extend(to_rns(h[0] * M % P))
    return g1, g2


def emit_header(path):
    L = LANES
    rows = []
    for i in range(30):
        rows.extend(L[i]["row"])
    l28 = []
    for i in range(30):
        l28.extend(L[i]["l28"])
    xi = [L[i]["xi"] for i in range(30)]
    aux = [L[i]["mpc"] if i < NB else L[i]["minv"] for i in range(30)]
    pm = [L[i]["pm"] for i in range(30)]
    kp = [L[i]["kp"] for i in range(30)]
    mods = [L[i]["m"] for i in range(30)]
    with open(path, "w") as f:
        f.write("// Generated by tools/gen_rns.py: RNS Montgomery constants (see bgv_rns.h).  Lane i < 15: base B,\n"
                "// i >= 15: base B'.  Do not edit.\n#pragma once\n#include <stdint.h>\n")
        f.write("#ifndef BGV_RNS_CONST\n#if defined(__HIP_DEVICE_COMPILE__)\n#define BGV_RNS_CONST static __constant__\n"
                "#else\n#define BGV_RNS_CONST static const\n#endif\n#endif\n")
        f.write("#define BGV_RNS_NB %d\n#define BGV_RNS_NL %d\n#define BGV_RNS_KNEG %d\n" % (NB, 2 * NB, KNEG))
        f.write("#define BGV_RNS_BETA_SHIFT %d\n#define BGV_RNS_BETA_ROUND 0x%xull\n" % (BETA_SHIFT, BETA_ROUND))
        f.write(c_array("kRnsMod", mods))
        f.write(c_array("kRnsXi", xi))    # B: -p^-1 M_i^-1; B': M'_j^-1
        f.write(c_array("kRnsXi2", [0 if i < NB else L[i]["minv"] * L[i]["xi"] % L[i]["m"] for i in range(30)]))  # B': M^-1 M'_j^-1
        f.write(c_array("kRnsAux", aux))  # B: -M' mod m_i; B': M^-1 mod m'_j
        f.write(c_array("kRnsPm", pm))    # p mod m
        f.write(c_array("kRnsKp", kp))    # K p mod m
        f.write(c_array("kRnsRow", rows))  # [lane][15]: B: |M'_j|_{m_i}; B': |M_k|_{m'_j}
        f.write(c_array("kRnsGBeta", GBETA))
        f.write(c_array("kRnsL28", l28))  # [lane][15]: 2^(28 k) mod m
        # constants in RNS M-form for conversions: in = M^2 / R28, out = R28 (see bgv_rns.h)
        f.write(c_array("kRnsCin", to_rns(M * M * pow(R28, -1, P) % P)))
        f.write(c_array("kRnsCout", to_rns(R28 % P)))
        g1, g2 = frob_consts()
        f.write(c_array("kRnsFrob1", g1))  # [k][re, im][lane]
        f.write(c_array("kRnsFrob2", g2))  # [k][lane]
        # integer reconstruction over base B (bgv_rns.h rns_to_fp): M_i^-1 mod m_i, G_i, M_i and M
        # in 28-bit limbs
        f.write(c_array("kRnsMinvB", [pow(M // m, -1, m) for m in BASE]))
        f.write(c_array("kRnsGB", [(1 << BETA_SHIFT) // m for m in BASE]))
        limbs = []
        for m in BASE:
            v = M // m
            limbs.extend([(v >> (LB * k)) & ((1 << LB) - 1) for k in range(15)])
        f.write(c_array("kRnsMiLimbs", limbs))  # [i][15]
        f.write(c_array("kRnsMLimbs", [(M >> (LB * k)) & ((1 << LB) - 1) for k in range(16)]))


if __name__ == "__main__":
    w = check()
    print("rns model ok: moduli 2^28 - c, c in [%d, %d]; M = 2^%.1f, M' = 2^%.1f; largest product output %.2f p"
          % ((1 << MB) - BASE[0], (1 << MB) - BASEP[-1], M.bit_length(), MP.bit_length(), w))
    if "--check" not in sys.argv:
        out = os.path.join(ROOT, "lodestar_amd", "csrc", "bgv_rns_consts.h")
        emit_header(out)
        print("wrote", out)
