"""Generates lodestar_amd/csrc/bgv_tmiller_prog.h: the twist-point half of the team Miller
loop as a table-driven program for a team of 16 lanes.

Every round is one instruction per lane: out = REDC(sum_k lin(A_k) * lin(B_k)), where a
lin() is a small integer combination of LDS slots plus K * p (K makes it non-negative) and
REDC is one Montgomery reduction of the double-width sum (bls_team.h wide_mac /
wide_redc).  The twist point T runs in HOMOGENEOUS projective coordinates (x = X/Z,
y = Y/Z; the Jacobian Q converted once), whose formulas need fewer rounds than
bls_pairing.h's Jacobian ones; the lines are the same lines up to Fp2 factors (2YZ for a
tangent, Z1 Z2^2 for a chord), which the final exponentiation kills, so the team loop's
pairing value equals miller_loop1's (tests/test_hostsim_math.py compares final_exp):

  init  (once per pair)  Q -> (QX QZ, QY, QZ^3) into bank 0 and the constants below  3 rounds
  dbl   2 rounds   R1: XY, B = Y^2, YZ, U = 3b'Z^2, A = X^2
                   R2: X3 = 2XY (B - 3U), Y3 = B (B + 6U) - 3U^2, Z3 = 8B YZ,
                       l0 = (B - U) Z_P^3, l1 = 3A (-X_P Z_P), l3 = 2YZ Y_P  (tangent x 2YZ)
  add   3 rounds   tools/gen_tcurve.py's projective addition with Q; u = Y2Z1 - Y1Z2,
                   v = X2Z1 - X1Z2 (Q = (X2, Y2, Z2)); R3 adds the chord
                       l0 = u X2 Z_P^3 - v Y2 Z_P^3, l1 = u Z2 (-X_P Z_P), l3 = v Z2 Y_P

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
# Q in homogeneous projective form (QPX, QY, QPZ) and the add lines' constants:
# X2Z = QPX Z_P^3, CX = QPZ (-X_P Z_P), CY = QPZ Y_P, Y2Z = QY Z_P^3
QPX, QPZ, X2Z, CX, CY = (9, 10), (11, 12), (13, 14), (15, 16), (17, 18)
BANK = [((19, 20), (21, 22), (23, 24)), ((25, 26), (27, 28), (29, 30))]  # T = (X, Y, Z)
L0, L1, L3 = (31, 32), (33, 34), (35, 36)   # the step's line
DUMMY = 37
ZP3 = 38                                    # Z_P^3 (lines scaled by it, bls_pairing.h miller_p)
Y2Z = (39, 40)
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
    QXp, QYp, QZp = pair(QX), pair(QY), pair(QZ)
    X0, Y0, Z0 = BANK[0]
    g.mul2(QXp, QZp, out=QPX)
    g.mul2(QXp, QZp, out=X0)
    g.ident2(QYp, Y0)
    zz = g.sqr2(QZp)
    g.mulfp(QYp, S(ZP3), out=Y2Z)
    g.new_round()
    g.mul2(QZp, zz, out=QPZ)
    g.mul2(QZp, zz, out=Z0)
    g.mulfp(pair(QPX), S(ZP3), out=X2Z)
    g.new_round()
    g.mulfp(pair(QPZ), S(XN), out=CX)
    g.mulfp(pair(QPZ), S(YP), out=CY)
    return g


def base_bounds(src_bank, init):
    b = dict(INPUT_BOUND)
    for s in QPX + QPZ + X2Z + CX + CY + Y2Z:
        b[s] = init.bound[s]
    for t in BANK[src_bank]:
        for s in t:
            b[s] = 2.0   # refreshed below from the producing programs (checked to be < 2)
    return b


def mul_b3(a):
    """3 b' a = 12 (1 + u) a (b' = 4 (1 + u), the twist's constant)"""
    return (scale(add(a[0], scale(a[1], -1)), 12), scale(add(a[0], a[1]), 12))


def neg_prod(c, d):
    """-(c d) as extra product terms of mul2 (re, im)"""
    return ([(scale(c[0], -1), d[0]), (c[1], d[1])], [(scale(c[0], -1), d[1]), (scale(c[1], -1), d[0])])


def prog_dbl(src, init, bank_bound):
    """T <- 2T over bank src -> bank 1 - src with the tangent line (projective)"""
    g = Prog("dbl%d" % src, {**base_bounds(src, init), **bank_bound})
    X, Y, Z = (pair(t) for t in BANK[src])
    X3o, Y3o, Z3o = BANK[1 - src]
    XY = g.mul2(X, Y)
    B = g.sqr2(Y)
    YZ = g.mul2(Y, Z)
    U = g.mul2(Z, mul_b3(Z))
    A = g.sqr2(X)
    g.new_round()
    g.mul2(lin2((2, XY)), lin2((1, B), (-3, U)), out=X3o)
    g.mul2(B, lin2((1, B), (6, U)), out=Y3o, extra=neg_prod(lin2((3, U)), U))
    g.mul2(lin2((8, B)), YZ, out=Z3o)
    g.mulfp(lin2((1, B), (-1, U)), S(ZP3), out=L0)
    g.mulfp(lin2((3, A)), S(XN), out=L1)
    g.mulfp(lin2((2, YZ)), S(YP), out=L3)
    return g


def prog_add(src, init, bank_bound):
    """T <- T + Q over bank src -> bank 1 - src with the chord line (projective)"""
    g = Prog("add%d" % src, {**base_bounds(src, init), **bank_bound})
    X1, Y1, Z1 = (pair(t) for t in BANK[src])
    X2, Y2, Z2 = pair(QPX), pair(QY), pair(QPZ)
    X3o, Y3o, Z3o = BANK[1 - src]
    A1 = g.mul2(Y2, Z1)
    A2 = g.mul2(Y1, Z2)
    B1 = g.mul2(X2, Z1)
    B2 = g.mul2(X1, Z2)
    ZZ = g.mul2(Z1, Z2)
    g.new_round()
    u = lin2((1, A1), (-1, A2))
    v = lin2((1, B1), (-1, B2))
    uu = g.sqr2(u)
    vv = g.sqr2(v)
    vZZ = g.mul2(v, ZZ)
    vB2 = g.mul2(v, B2)
    uB2 = g.mul2(u, B2)
    uZZ = g.mul2(u, ZZ)
    uv = g.mul2(u, v)
    vA2 = g.mul2(v, A2)
    g.new_round()
    g.mul2(uu, vZZ, out=X3o, extra=neg_prod(vv, lin2((1, vv), (2, vB2))))
    g.mul2(vv, lin2((3, uB2), (1, uv), (-1, vA2)), out=Y3o, extra=neg_prod(uu, uZZ))
    g.mul2(vv, vZZ, out=Z3o)
    g.mul2(u, pair(X2Z), out=L0, extra=neg_prod(v, pair(Y2Z)))
    g.mul2(u, pair(CX), out=L1)
    g.mul2(v, pair(CY), out=L3)
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
