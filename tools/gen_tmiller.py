"""Generates lodestar_amd/csrc/bgv_tmiller_prog.h: the twist-point half of the team Miller
loop as a table-driven program for a team of 16 lanes.

Every round is one instruction per lane: out = REDC(sum_k lin(A_k) * lin(B_k)), where a
lin() is a small integer combination of LDS slots plus K * p (K makes it non-negative) and
REDC is one Montgomery reduction of the double-width sum (bls_team.h wide_mac /
wide_redc).  The rounds restate bls_pairing.h exactly (same formulas, same line scaling),
so the team loop's Fp12 value equals miller_loop1's:

  init  (once per pair)  miller_jq_make: zz = Z2^2, xz = X2 Z2, zzz = Z2^3, zzz*xn, zzz*yp
  dbl   3 rounds         miller_dbl: T <- 2T, line (l0, l1, l3)
  add   5 rounds         miller_add_jq: T <- T + Q, line

The generator tracks an upper bound (in units of p) for every slot and checks each
instruction against the reduction's input range, so no lin() or sum can leave the
representation (limbs < 2^28, value < 2^392, column sums < 2^63).

    python tools/gen_tmiller.py    # rewrites the header
"""
import os
from fractions import Fraction

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F624_1EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R_OVER_P = Fraction(2 ** 392, P)
LANES = 16
MAX_TERMS = 8      # products per instruction (column sums < 2^63 for limbs < 2^28)
MAX_LIN = 6        # slots per lin()

# ---- fixed slots --------------------------------------------------------------------------
ONE, XN, YP = 0, 1, 2                       # Montgomery 1, -X_P Z_P, Y_P (P Jacobian)
QX, QY, QZ = (3, 4), (5, 6), (7, 8)         # Q (Jacobian)
ZZ, XZ, ZZZ, ZZZ_XN, ZZZ_YP = (9, 10), (11, 12), (13, 14), (15, 16), (17, 18)
BANK = [((19, 20), (21, 22), (23, 24)), ((25, 26), (27, 28), (29, 30))]  # T = (X, Y, Z)
L0, L1, L3 = (31, 32), (33, 34), (35, 36)   # the step's line
DUMMY = 37
ZP3 = 38                                    # Z_P^3 (lines scaled by it, bls_pairing.h miller_p)
Y2S = (39, 40)                              # Y2 Z_P^3
TEMP0 = 41

INPUT_BOUND = {ONE: 1, XN: 2, YP: 2, ZP3: 2}
for s in QX + QY + QZ:
    INPUT_BOUND[s] = 2


def form(*pairs):
    f = {}
    for s, c in pairs:
        f[s] = f.get(s, 0) + c
    return {s: c for s, c in f.items() if c}


def add(*fs):
    out = {}
    for f in fs:
        for s, c in f.items():
            out[s] = out.get(s, 0) + c
    return {s: c for s, c in out.items() if c}


def scale(f, k):
    return {s: c * k for s, c in f.items()}


def sub(a, b):
    return add(a, scale(b, -1))


def S(s):
    return {s: 1}


class Prog:
    def __init__(self, name, bounds):
        self.name = name
        self.bound = dict(bounds)      # slot -> upper bound in units of p
        self.written = {s: -1 for s in bounds}
        self.rounds = [[]]
        self.next_temp = TEMP0
        self.reads = {}

    def check(self):
        # no slot is both written and read in one round (lanes of a round run concurrently)
        for r, rnd in enumerate(self.rounds):
            outs = {o for o, _ in rnd}
            assert not (outs & self.reads.get(r, set())), (self.name, r, outs & self.reads.get(r, set()))

    def new_round(self):
        self.rounds.append([])

    def _lin(self, f):
        assert 0 < len(f) <= MAX_LIN, (self.name, f)
        r = len(self.rounds) - 1
        for s in f:
            assert s in self.written and self.written[s] < r, (self.name, "slot %d not ready in round %d" % (s, r))
        neg = sum(-c * self.bound[s] for s, c in f.items() if c < 0)
        K = int(-(-neg // 1))
        upper = sum(c * self.bound[s] for s, c in f.items() if c > 0) + K
        assert upper < 1024, (self.name, f, upper)
        return (sorted(f.items()), K, upper)

    def op(self, terms, out=None):
        """out = REDC(sum a_k * b_k); terms: [(form_a, form_b), ...]; returns {out: 1}"""
        assert 0 < len(terms) <= MAX_TERMS
        lins, acc = [], 0
        for a, b in terms:
            la, lb = self._lin(a), self._lin(b)
            lins.append((la, lb))
            acc += la[2] * lb[2]
        assert acc < R_OVER_P * Fraction(9, 10), (self.name, acc)
        if out is None:
            out = self.next_temp
            self.next_temp += 1
        r = len(self.rounds) - 1
        assert self.written.get(out, -2) < r, (self.name, "slot %d written twice in a round" % out)
        self.reads.setdefault(r, set()).update(s for la, lb in lins for s, _ in la[0] + lb[0])
        self.rounds[-1].append((out, lins))
        assert len(self.rounds[-1]) <= LANES, (self.name, "round too wide")
        self.bound[out] = float(Fraction(acc) / R_OVER_P) + 1.0
        self.written[out] = r
        return S(out)

    # Fp2 helpers on (form, form)
    def sqr2(self, a, out=(None, None)):
        """(a0 + a1)(a0 - a1), 2 a0 a1 -- fp2_sqr"""
        a0, a1 = a
        return (self.op([(add(a0, a1), sub(a0, a1))], out[0]), self.op([(scale(a0, 2), a1)], out[1]))

    def mul2(self, a, b, out=(None, None), extra=((), ())):
        """a * b (schoolbook per component, one reduction each) plus extra product terms"""
        a0, a1 = a
        b0, b1 = b
        re = [(a0, b0), (scale(a1, -1), b1)] + list(extra[0])
        im = [(a0, b1), (a1, b0)] + list(extra[1])
        return (self.op(re, out[0]), self.op(im, out[1]))

    def mulfp(self, a, k, out=(None, None)):
        return (self.op([(a[0], k)], out[0]), self.op([(a[1], k)], out[1]))

    def ident2(self, a, out):
        return (self.op([(a[0], S(ONE))], out[0]), self.op([(a[1], S(ONE))], out[1]))


def pair(t):
    return (S(t[0]), S(t[1]))


def lin2(*terms):
    """sum of c * (Fp2 pair) -> pair of forms"""
    re = add(*[scale(p[0], c) for c, p in terms])
    im = add(*[scale(p[1], c) for c, p in terms])
    return (re, im)


def prog_init():
    g = Prog("init", INPUT_BOUND)
    Q = {"x": pair(QX), "y": pair(QY), "z": pair(QZ)}
    zz = g.sqr2(Q["z"], out=ZZ)
    xz = g.mul2(Q["x"], Q["z"])
    g.mulfp(Q["y"], S(ZP3), out=Y2S)
    g.new_round()
    zzz = g.mul2(zz, Q["z"], out=ZZZ)
    g.mulfp(xz, S(ZP3), out=XZ)
    g.new_round()
    g.mulfp(zzz, S(XN), out=ZZZ_XN)
    g.mulfp(zzz, S(YP), out=ZZZ_YP)
    return g


def base_bounds(src_bank, init):
    b = dict(INPUT_BOUND)
    for s in ZZ + XZ + ZZZ + ZZZ_XN + ZZZ_YP + Y2S:
        b[s] = init.bound[s]
    for t in BANK[src_bank]:
        for s in t:
            b[s] = 2.0   # refreshed below from the producing programs (checked to be < 2)
    return b


def prog_dbl(src, init, bank_bound):
    """miller_dbl (bls_pairing.h:11-28) over bank src -> bank 1 - src"""
    g = Prog("dbl%d" % src, {**base_bounds(src, init), **bank_bound})
    X, Y, Z = (pair(t) for t in BANK[src])
    X3o, Y3o, Z3o = BANK[1 - src]
    # R1: A = X^2, B = Y^2, ZZ = Z^2, Z3 = (Y + Z)^2 - B - ZZ = 2 Y Z
    A = g.sqr2(X)
    B = g.sqr2(Y)
    ZZl = g.sqr2(Z)
    Z3 = g.mul2(lin2((2, Y)), Z, out=Z3o)
    g.new_round()
    # R2: C = B^2, G = (X + B)^2, F = E^2 (E = 3A), l0 = E X - 2B, EZZ = E ZZ, Z3ZZ = Z3 ZZ
    C = g.sqr2(B)
    G = g.sqr2(lin2((1, X), (1, B)))
    F = g.sqr2(lin2((3, A)))
    E = lin2((3, A))
    EX = g.mul2(E, X)
    EZZ = g.mul2(E, ZZl)
    Z3ZZ = g.mul2(Z3, ZZl)
    g.new_round()
    # R3: D = 2(G - A - C); X3 = F - 2D; Y3 = E (D - X3) - 8C; l1 = EZZ xn; l3 = Z3ZZ yp
    D = lin2((2, G), (-2, A), (-2, C))
    X3 = lin2((1, F), (-4, G), (4, A), (4, C))
    g.ident2(X3, X3o)
    DmX3 = lin2((6, G), (-6, A), (-6, C), (-1, F))
    negC8 = lin2((-8, C))
    g.mul2(E, DmX3, out=Y3o, extra=([(negC8[0], S(ONE))], [(negC8[1], S(ONE))]))
    g.mulfp(EZZ, S(XN), out=L1)
    g.mulfp(Z3ZZ, S(YP), out=L3)
    g.mulfp(lin2((1, EX), (-2, B)), S(ZP3), out=L0)   # (E X - 2B) Z_P^3
    del D
    return g


def prog_add(src, init, bank_bound):
    """miller_add_jq (bls_pairing.h:99-120) over bank src -> bank 1 - src"""
    g = Prog("add%d" % src, {**base_bounds(src, init), **bank_bound})
    X, Y, Z = (pair(t) for t in BANK[src])
    X3o, Y3o, Z3o = BANK[1 - src]
    q = {"x": pair(QX), "y": pair(QY), "z": pair(QZ)}
    zz, xz, zzz, zzz_xn, zzz_yp = pair(ZZ), pair(XZ), pair(ZZZ), pair(ZZZ_XN), pair(ZZZ_YP)
    # R1: ZZ = Z^2, U1 = X zz, S1 = Y zz Z2 (= Y zzz), Z3' = (Z + Z2)^2 - ZZ - zz = 2 Z Z2, Y2Z = Y2 Z
    ZZl = g.sqr2(Z)
    U1 = g.mul2(X, zz)
    S1 = g.mul2(Y, zzz)
    Z3p = g.mul2(lin2((2, Z)), q["z"])
    Y2Z = g.mul2(q["y"], Z)
    g.new_round()
    # R2: U2 = X2 ZZ, S2 = Y2 Z ZZ
    U2 = g.mul2(q["x"], ZZl)
    S2 = g.mul2(Y2Z, ZZl)
    g.new_round()
    # R3: H = U2 - U1, HH = H^2, r = 2(S2 - S1), rr = r^2, Z3 = Z3' H
    H = lin2((1, U2), (-1, U1))
    r = lin2((2, S2), (-2, S1))
    HH = g.sqr2(H)
    rr = g.sqr2(r)
    Z3 = g.mul2(Z3p, H, out=Z3o)
    g.new_round()
    # R4: J = H I = 4 H HH, V = U1 I = 4 U1 HH, l0 = r xz - Y2 Z3 (xz, Y2 scaled by Z_P^3),
    # l1 = r zzz_xn, l3 = Z3 zzz_yp
    J = g.mul2(lin2((4, H)), HH)
    V = g.mul2(lin2((4, U1)), HH)
    y2s = pair(Y2S)
    nY2 = lin2((-1, y2s))
    g.mul2(r, xz, out=L0, extra=([(nY2[0], Z3[0]), (y2s[1], Z3[1])],
                                 [(nY2[0], Z3[1]), (nY2[1], Z3[0])]))
    g.mul2(r, zzz_xn, out=L1)
    g.mul2(Z3, zzz_yp, out=L3)
    g.new_round()
    # R5: X3 = r^2 - J - 2V, Y3 = r (V - X3) - 2 S1 J
    X3 = lin2((1, rr), (-1, J), (-2, V))
    g.ident2(X3, X3o)
    VmX3 = lin2((3, V), (-1, rr), (1, J))
    nS1 = lin2((-2, S1))
    # -2 S1 J = (-2 S1_0 J_0 + 2 S1_1 J_1) + (-2 S1_0 J_1 - 2 S1_1 J_0) u
    g.mul2(r, VmX3, out=Y3o, extra=([(nS1[0], J[0]), (scale(S1[1], 2), J[1])],
                                    [(nS1[0], J[1]), (nS1[1], J[0])]))
    return g


def emit(progs):
    """Flat byte table: per program a header {nrounds}, per round {T, M, lanes}, per lane
    {out, then T x (A: M x (idx, coef), K; B: M x (idx, coef), K)} (unused terms: coef 0)."""
    lines = []
    table = []
    offsets = {}
    for g in progs:
        offsets[g.name] = len(table)
        table.append(len(g.rounds))
        for rnd in g.rounds:
            T = max(len(l) for _, l in rnd)
            M = max(max(len(a[0]), len(b[0])) for _, l in rnd for a, b in l)
            table += [T, M]
            for lane in range(LANES):
                if lane < len(rnd):
                    out, lins = rnd[lane]
                else:
                    out, lins = DUMMY, []
                table.append(out)
                for k in range(T):
                    for side in (0, 1):
                        if k < len(lins):
                            items, K, _ = lins[k][side]
                        else:
                            items, K = [], 0
                        for j in range(M):
                            if j < len(items):
                                s, c = items[j]
                                assert -128 <= c < 128
                                table += [s, c & 0xff]
                            else:
                                table += [ONE, 0]
                        table.append(K)
    nslots = max(max(g.next_temp for g in progs), TEMP0)
    lines.append("// GENERATED by tools/gen_tmiller.py -- do not edit.")
    lines.append("// Team Miller loop twist-point programs (see the generator's docstring).")
    lines.append("#pragma once")
    lines.append("#define TMP_NSLOT %d" % nslots)
    for name, off in offsets.items():
        lines.append("#define TMP_%s %d" % (name.upper(), off))
    for name, val in (("ONE", ONE), ("XN", XN), ("YP", YP), ("QX", QX[0]), ("QY", QY[0]), ("QZ", QZ[0]),
                      ("BANK0", BANK[0][0][0]), ("BANK1", BANK[1][0][0]), ("L0", L0[0]), ("L1", L1[0]),
                      ("L3", L3[0]), ("DUMMY", DUMMY), ("ZP3", ZP3)):
        lines.append("#define TMP_S_%s %d" % (name, val))
    lines.append("#define TMP_TABLE_BYTES %d" % len(table))
    body = ",".join(str(b) for b in table)
    lines.append("#define TMP_TABLE_INIT {%s}" % body)
    worst = max((max(len(r) for r in g.rounds), g.name) for g in progs)
    lines.append("// widest round: %d lanes (%s); rounds: %s" % (worst[0], worst[1],
                 ", ".join("%s %d" % (g.name, len(g.rounds)) for g in progs)))
    return "\n".join(lines) + "\n"


def main():
    init = prog_init()
    bank_bound = {}
    # state bounds: outputs of ident / mul2 rounds, iterate to a fixed point
    for it in range(4):
        progs = [init]
        bb = {}
        for src in (0, 1):
            b = {s: bank_bound.get(s, 2.0) for t in BANK[src] for s in t}
            progs.append(prog_dbl(src, init, b))
            progs.append(prog_add(src, init, b))
        nb = {}
        for g in progs[1:]:
            for t in BANK[0] + BANK[1]:
                for s in t:
                    if s in g.bound and g.written.get(s, -1) >= 0:
                        nb[s] = max(nb.get(s, 0), g.bound[s])
        for s in nb:
            nb[s] = max(nb[s], 2.0)
        if nb == bank_bound:
            break
        bank_bound = nb
    for g in progs:
        g.check()
        for s in L0 + L1 + L3:
            if g.written.get(s, -1) >= 0:
                assert g.bound[s] < 1.5, (g.name, s, g.bound[s])  # lines feed tm_mul_line_lane
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lodestar_amd", "csrc",
                       "bgv_tmiller_prog.h")
    open(out, "w").write(emit(progs))
    print("wrote", out, "slots", max(g.next_temp for g in progs))


if __name__ == "__main__":
    main()
