"""Lane-level emulation of the wave-cooperative Fp products (lodestar_amd/csrc/bgv_wfp.h
wfp_mul3 / wfp_umul_l, bgv_wround.h wr_instr) -- test infrastructure.

A wavefront is a list of 64 lane values; the DPP moves, readlane and ballot are the list
operations below, and every 32/64-bit intermediate wraps exactly as the device's registers do.
The emulation follows the kernels statement by statement, so a CPU test can check the algorithms
(rotated operands, the reduction as two more products, the carry passes, the ballot carry
lookahead) against plain Montgomery arithmetic; the GPU checks the compiled code against
fp_mul_body (tools/ubench_wfp.hip, tools/ubench_wround.hip).

    python tools/emu_wfp.py [cases]
"""
import random
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
NL, LB, MASK = 14, 28, (1 << 28) - 1
R = 1 << (LB * NL)
NP = (-pow(P, -1, R)) % R
N0 = NP & MASK
W = 64
M32, M64 = (1 << 32) - 1, (1 << 64) - 1
PL = [(P >> (LB * i)) & MASK for i in range(NL)]
NPL = [(NP >> (LB * i)) & MASK for i in range(NL)]


def limbs(x):
    return [(x >> (LB * i)) & MASK for i in range(NL)]


def value(v):  # lanes 0..13 as limbs (any magnitude)
    return sum(int(v[l]) << (LB * l) for l in range(NL))


def rol1(v):  # lane L reads lane L + 1 (mod 64)
    return [v[(L + 1) % W] for L in range(W)]


def ror1(v):  # lane L reads lane L - 1 (mod 64)
    return [v[(L - 1) % W] for L in range(W)]


def shr1(v):  # lane L reads lane L - 1, lane 0 reads 0
    return [0] + v[:-1]


def ballot(c):
    return sum(1 << L for L in range(W) if c[L])


def u32(x):
    return x & M32


def u64(x):
    return x & M64


def s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def from_limbs(x):  # wfp_from: limb l in lane l
    return [x[L] if L < NL else 0 for L in range(W)]


def wfp_mul3(a, b):
    """bgv_wfp.h wfp_mul3 (a, b: 64 lane u32 values, limbs < 2^29 in lanes 0..13)"""
    prot = []
    r = [PL[L] if L < NL else 0 for L in range(W)]
    rots = [None] * NL
    for k in range(1, NL + 1):
        r = rol1(r)
        rots[NL - k] = r
    prot = rots
    nrot = [None] * NL
    r = [NPL[L] if L < NL else 0 for L in range(W)]
    for k in range(1, NL + 1):
        r = rol1(r)
        nrot[NL - k] = r
    br = [None] * NL
    r = list(b)
    for k in range(1, NL + 1):
        r = rol1(r)
        br[NL - k] = r
    T = [0] * W
    for i in range(NL - 1, -1, -1):
        ai = a[i]
        T = [u64(T[L] + ai * br[i][L]) for L in range(W)]
    # t = T mod R (lanes 50..63)
    h = [x >> LB for x in T]
    hs = [(shr1([u32(x >> 32) for x in h])[L] << 32) | shr1([u32(x) for x in h])[L] for L in range(W)]
    v1 = [u64((T[L] & MASK) + hs[L]) for L in range(W)]
    t = [u32((v1[L] & MASK) + shr1([u32(x >> LB) for x in v1])[L]) for L in range(W)]
    M = [0] * W
    for i in range(NL):
        ti = t[50 + i]
        M = [u64(M[L] + ti * nrot[i][L]) for L in range(W)]
    h = [x >> LB for x in M]
    hs = [(shr1([u32(x >> 32) for x in h])[L] << 32) | shr1([u32(x) for x in h])[L] for L in range(W)]
    v1 = [u64((M[L] & MASK) + hs[L]) for L in range(W)]
    m = [u32((v1[L] & MASK) + shr1([u32(x >> LB) for x in v1])[L]) for L in range(W)]
    for i in range(NL):
        mi = m[50 + i]
        T = [u64(T[L] + mi * prot[i][L]) for L in range(W)]
    h = [x >> LB for x in T]
    hs = [(ror1([u32(x >> 32) for x in h])[L] << 32) | ror1([u32(x) for x in h])[L] for L in range(W)]
    v1 = [u64((T[L] & MASK) + hs[L]) for L in range(W)]
    v2 = [u32((v1[L] & MASK) + ror1([u32(x >> LB) for x in v1])[L]) for L in range(W)]
    low = ballot([x != 0 for x in v2]) & 0xFFFC000000000000
    res = [u32(v2[L] + (1 if (L == 0 and low) else 0)) for L in range(W)]
    return [res[L] if L < NL else 0 for L in range(W)]


def wfp_umul(a_limbs, b_limbs):
    """bgv_wfp.h wfp_umul_l (uniform operands): returns the 14 normalized limbs of wfp_to"""
    lane = list(range(W))
    low = [L >= 50 for L in lane]
    r = from_limbs(b_limbs)
    br = [None] * NL
    for k in range(1, NL + 1):
        r = rol1(r)
        br[NL - k] = r
    T = [0] * W
    for i in range(NL - 1, -1, -1):
        T = [u64(T[L] + a_limbs[i] * br[i][L]) for L in range(W)]
    h = [x >> LB for x in T]
    hs = [(shr1([u32(x >> 32) for x in h])[L] << 32) | shr1([u32(x) for x in h])[L] for L in range(W)]
    v1 = [u64((T[L] & MASK) + hs[L]) for L in range(W)]
    t = [u32((v1[L] & MASK) + shr1([u32(x >> LB) for x in v1])[L]) for L in range(W)]
    t = [t[L] if low[L] else 0 for L in range(W)]
    M = [u64(NPL[0] * x) for x in t]
    tr = t
    for j in range(1, NL):
        tr = ror1(tr)
        M = [u64(M[L] + NPL[j] * tr[L]) for L in range(W)]
    h = [x >> LB for x in M]
    hs = [(shr1([u32(x >> 32) for x in h])[L] << 32) | shr1([u32(x) for x in h])[L] for L in range(W)]
    v1 = [u64((M[L] & MASK) + hs[L]) for L in range(W)]
    m = [u32((v1[L] & MASK) + shr1([u32(x >> LB) for x in v1])[L]) for L in range(W)]
    m = [m[L] if low[L] else 0 for L in range(W)]
    mr = m
    T = [u64(T[L] + PL[0] * mr[L]) for L in range(W)]
    for j in range(1, NL):
        mr = ror1(mr)
        T = [u64(T[L] + PL[j] * mr[L]) for L in range(W)]
    h = [x >> LB for x in T]
    hs = [(ror1([u32(x >> 32) for x in h])[L] << 32) | ror1([u32(x) for x in h])[L] for L in range(W)]
    v1 = [u64((T[L] & MASK) + hs[L]) for L in range(W)]
    v2 = [u32((v1[L] & MASK) + ror1([u32(x >> LB) for x in v1])[L]) for L in range(W)]
    lowbits = ballot([x != 0 for x in v2]) & 0xFFFC000000000000
    res = [u32(v2[L] + (1 if (L == 0 and lowbits) else 0)) for L in range(W)]
    # wfp_to: readlanes and one carry chain
    out, c = [], 0
    for l in range(NL - 1):
        s = u32(res[l] + c)
        out.append(s & MASK)
        c = s >> LB
    out.append(u32(res[NL - 1] + c))
    return out


# ---- bgv_wround.h (signed operand digits, exact resolution) --------------------------------
def shr64(v):
    return [0] + v[:-1]


def ror64(v):
    return [v[-1]] + v[:-1]


def pass_(x):
    return [(x[L] & MASK) + (shr64([y >> LB for y in x])[L]) for L in range(W)]


def pass_ring(x):
    return [(x[L] & MASK) + (ror64([y >> LB for y in x])[L]) for L in range(W)]


def carries(G, Pm, rng):
    G &= rng
    Pm &= rng
    X = G | Pm
    S = X + G
    C = (S ^ X ^ G) & M64
    top = rng & ~(rng >> 1)
    top_out = (S >> 64) & 1 if top == 1 << 63 else int(bool(C & (top << 1)))
    return C & rng, bool(top_out)


def resolve(d, rng):
    inn = [(rng >> L) & 1 for L in range(W)]
    is_top = [inn[L] and not ((rng >> L) & 2) for L in range(W)]
    C, top = carries(ballot([inn[L] and d[L] >= 1 << LB for L in range(W)]),
                     ballot([inn[L] and d[L] == MASK for L in range(W)]), rng)
    e = []
    for L in range(W):
        ci = (C >> L) & 1
        co = top if is_top[L] else (inn[L] and (C >> (L + 1)) & 1)
        e.append(d[L] + ci - ((1 << LB) if co else 0))
    C, btop = carries(ballot([inn[L] and e[L] < 0 for L in range(W)]),
                      ballot([inn[L] and e[L] == 0 for L in range(W)]), rng)
    f = []
    for L in range(W):
        bi = (C >> L) & 1
        bo = btop if is_top[L] else (inn[L] and (C >> (L + 1)) & 1)
        f.append(e[L] - bi + ((1 << LB) if bo else 0))
    return [f[L] if inn[L] else 0 for L in range(W)], int(top) - int(btop)


def wr_lin(slots, terms, K):
    """terms: [(slot limbs, coefficient)]; returns signed digits in [-1, 2^28]"""
    acc = [(K * PL[L] if L < NL else 0) for L in range(W)]
    for x, cf in terms:
        acc = [acc[L] + (cf * x[L] if L < NL else 0) for L in range(W)]
    acc = pass_(pass_(acc))
    return [acc[L] if L < NL else 0 for L in range(W)]


def wr_mac(col, a, b):
    br = [None] * NL
    r = list(b)
    for k in range(1, NL + 1):
        r = rol1(r)
        br[NL - k] = r
    for i in range(NL - 1, -1, -1):
        col = [col[L] + a[i] * br[i][L] for L in range(W)]
    return col


def wr_reduce(col):
    LOW, HIGH = 0xFFFC000000000000, 0x3FFF
    for L in range(W):
        assert -(1 << 63) <= col[L] < 1 << 63
    t2 = pass_(pass_(pass_(col)))
    t, _ = resolve(t2, LOW)
    M = [NPL[0] * t[L] for L in range(W)]
    tr = t
    for j in range(1, NL):
        tr = ror1(tr)
        M = [M[L] + NPL[j] * tr[L] for L in range(W)]
    M = [u64(x) for x in M]
    h = [x >> LB for x in M]
    hs = [(shr1([u32(x >> 32) for x in h])[L] << 32) | shr1([u32(x) for x in h])[L] for L in range(W)]
    v1 = [u64((M[L] & MASK) + hs[L]) for L in range(W)]
    m = [u32((v1[L] & MASK) + shr1([u32(x >> LB) for x in v1])[L]) for L in range(W)]
    m = [m[L] if L >= 50 else 0 for L in range(W)]
    mr = m
    U = [col[L] + PL[0] * mr[L] for L in range(W)]
    for j in range(1, NL):
        mr = ror1(mr)
        U = [U[L] + PL[j] * mr[L] for L in range(W)]
    for L in range(W):
        assert -(1 << 63) <= U[L] < 1 << 63
    U = pass_ring(pass_ring(pass_ring(U)))
    _, cl = resolve(U, LOW)
    hi = [U[L] + (cl if L == 0 else 0) for L in range(W)]
    out, _ = resolve(hi, HIGH)
    return out


def check(cases=40, seed=1):
    rng = random.Random(seed)
    rinv = pow(R, -1, P)
    for n in range(cases):
        # operands < 4p with limbs < 2^29 (fp_mul's contract): a normalized value plus a
        # limb-wise sum for the redundant case
        x = rng.randrange(2 * P)
        y = rng.randrange(2 * P)
        xa = limbs(x)
        ya = limbs(y)
        if n % 3 == 1:
            z = rng.randrange(2 * P)
            xa = [u + v for u, v in zip(limbs(x), limbs(z))]
            x = x + z
        got = wfp_mul3(from_limbs(xa), from_limbs(ya))
        assert all(0 <= g < 1 << 29 for g in got[:NL]) and not any(got[NL:]), "limb bounds"
        assert value(got) % P == x * y * rinv % P, "wfp_mul3 value"
        assert value(got) < 2 * P, "wfp_mul3 weakly reduced"
        u = wfp_umul(limbs(x % (2 * P)), ya)
        assert value(u) == value(got) if n % 3 != 1 else value(u) % P == value(got) % P
        assert all(v < 1 << LB for v in u[:NL - 1]) and value(u) < 2 * P, "wfp_umul normalized"
        # wr_instr: REDC(lin(A) lin(B) + lin(C) lin(D)) with signed coefficients
        s = [rng.randrange(2 * P) for _ in range(4)]
        sl = [limbs(v) for v in s]
        A = wr_lin(sl, [(sl[0], 1), (sl[1], -2)], 4)
        B = wr_lin(sl, [(sl[2], 3)], 0)
        C = wr_lin(sl, [(sl[3], 1)], 0)
        D = wr_lin(sl, [(sl[0], -1), (sl[2], 1)], 2)
        la = s[0] - 2 * s[1] + 4 * P
        lb = 3 * s[2]
        lc = s[3]
        ld = -s[0] + s[2] + 2 * P
        for dig, want in ((A, la), (B, lb), (C, lc), (D, ld)):
            assert value([int(v) for v in dig]) == want and all(-1 <= v <= 1 << LB for v in dig[:NL])
        col = wr_mac(wr_mac([0] * W, A, B), C, D)
        out = wr_reduce(col)
        want = (la * lb + lc * ld) * rinv % P
        assert all(0 <= v < 1 << LB for v in out[:NL]), "wr_instr normalized"
        assert value(out) % P == want, "wr_instr value"
        assert value(out) < 2 * P or (la * lb + lc * ld) >= 4 * P * P
    return cases


if __name__ == "__main__":
    n = check(int(sys.argv[1]) if len(sys.argv) > 1 else 40)
    print("emulated wfp_mul3 / wfp_umul / wr_instr == Montgomery products: %d cases" % n)
