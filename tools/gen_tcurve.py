"""Generates lodestar_amd/csrc/bgv_tcurve_prog.h: G2 point programs for a team of 16 lanes
(the latency path's cofactor clearing and r * sig, bgv_tcurve.h).

Same instruction model as tools/gen_tmiller.py (one Fp output per lane per round,
REDC(sum_k lin(A_k) lin(B_k)), bounds tracked per slot), over fixed point "banks" of six
Fp slots (X, Y, Z as Fp2 pairs).  Programs restate bls_curve.h:

  dbl45 / dbl54   jac_dbl (dbl-2009-l), bank 4 -> 5 and 5 -> 4      3 rounds
  add405 / add504 jac_add_raw (add-2007-bl), bank 4|5 + bank 0      5 rounds
  add123          jac_add_raw, bank 1 + bank 2 -> bank 3            5 rounds
  psi12           g2_psi: (conj(X) cx, conj(Y) cy, conj(Z)), 1 -> 2  1 round
  psi2_12         g2_psi2: (X c, Y c', Z), 1 -> 2                     1 round

Additions are the generic-case formulas; the driver checks H != 0 (slot TCP_S_HH of the
add programs) and falls back to the complete one-lane formulas if it ever is.

    python tools/gen_tcurve.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_tmiller as gm  # noqa: E402
from gen_tmiller import Prog, S, add, lin2, pair, scale  # noqa: E402

ONE = 0
PSI_CX, PSI_CY = (1, 2), (3, 4)
PSI2_CX, PSI2_CY = 5, 6
DUMMY = 7
NBANK = 10
BANK0 = 8


def bank(k):
    b = BANK0 + 6 * k
    return ((b, b + 1), (b + 2, b + 3), (b + 4, b + 5))


TEMP0 = BANK0 + 6 * NBANK
gm.TEMP0 = TEMP0  # Prog allocates temporaries from here
gm.ONE = ONE
gm.DUMMY = DUMMY

BOUND_IN = {ONE: 1, PSI_CX[0]: 1, PSI_CX[1]: 1, PSI_CY[0]: 1, PSI_CY[1]: 1, PSI2_CX: 1, PSI2_CY: 1}
PT_BOUND = 2.0  # every bank value is weakly reduced (< 2p): checked on every program's outputs


def bounds_with(*banks):
    b = dict(BOUND_IN)
    for k in banks:
        for t in bank(k):
            for s in t:
                b[s] = PT_BOUND
    return b


def prog_dbl(src, dst):
    g = Prog("dbl%d%d" % (src, dst), bounds_with(src))
    X, Y, Z = (pair(t) for t in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    A = g.sqr2(X)
    B = g.sqr2(Y)
    g.mul2(lin2((2, Y)), Z, out=Z3o)  # Z3 = 2 Y Z
    g.new_round()
    C = g.sqr2(B)
    G = g.sqr2(lin2((1, X), (1, B)))
    F = g.sqr2(lin2((3, A)))
    g.new_round()
    # X3 = F - 2D, D = 2(G - A - C);  Y3 = E (D - X3) - 8C, E = 3A
    g.ident2(lin2((1, F), (-4, G), (4, A), (4, C)), X3o)
    E = lin2((3, A))
    DmX3 = lin2((6, G), (-6, A), (-6, C), (-1, F))
    nC8 = lin2((-8, C))
    g.mul2(E, DmX3, out=Y3o, extra=([(nC8[0], S(ONE))], [(nC8[1], S(ONE))]))
    return g


HH_SLOTS = {}


def prog_add(a, b, dst):
    g = Prog("add%d%d%d" % (a, b, dst), bounds_with(a, b))
    X1, Y1, Z1 = (pair(t) for t in bank(a))
    X2, Y2, Z2 = (pair(t) for t in bank(b))
    X3o, Y3o, Z3o = bank(dst)
    # R1: Z1Z1, Z2Z2, Y1 Z2, Y2 Z1, Zs = (Z1 + Z2)^2 - Z1Z1 - Z2Z2 = 2 Z1 Z2
    Z1Z1 = g.sqr2(Z1)
    Z2Z2 = g.sqr2(Z2)
    Y1Z2 = g.mul2(Y1, Z2)
    Y2Z1 = g.mul2(Y2, Z1)
    Zs = g.mul2(lin2((2, Z1)), Z2)
    g.new_round()
    # R2: U1 = X1 Z2Z2, U2 = X2 Z1Z1, S1 = Y1 Z2 Z2Z2, S2 = Y2 Z1 Z1Z1
    U1 = g.mul2(X1, Z2Z2)
    U2 = g.mul2(X2, Z1Z1)
    S1 = g.mul2(Y1Z2, Z2Z2)
    S2 = g.mul2(Y2Z1, Z1Z1)
    g.new_round()
    # R3: H = U2 - U1, HH = H^2, r = 2(S2 - S1), rr = r^2, Z3 = Zs H
    H = lin2((1, U2), (-1, U1))
    r = lin2((2, S2), (-2, S1))
    HH = g.sqr2(H)
    rr = g.sqr2(r)
    g.mul2(Zs, H, out=Z3o)
    g.new_round()
    # R4: I = 4 HH, J = H I, V = U1 I
    J = g.mul2(lin2((4, H)), HH)
    V = g.mul2(lin2((4, U1)), HH)
    g.new_round()
    # R5: X3 = rr - J - 2V, Y3 = r (V - X3) - 2 S1 J
    g.ident2(lin2((1, rr), (-1, J), (-2, V)), X3o)
    VmX3 = lin2((3, V), (-1, rr), (1, J))
    nS1 = lin2((-2, S1))
    g.mul2(r, VmX3, out=Y3o, extra=([(nS1[0], J[0]), (scale(S1[1], 2), J[1])],
                                    [(nS1[0], J[1]), (nS1[1], J[0])]))
    HH_SLOTS[g.name] = (list(HH[0])[0], list(HH[1])[0])
    return g


def prog_psi(src, dst):
    """psi(P) = (conj(X) cx, conj(Y) cy, conj(Z)), bls_curve.h g2_psi"""
    g = Prog("psi%d%d" % (src, dst), bounds_with(src))
    X, Y, Z = (pair(t) for t in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    for (v0, v1), (c0, c1), out in ((X, PSI_CX, X3o), (Y, PSI_CY, Y3o)):
        # (v0 - v1 u)(c0 + c1 u) = (v0 c0 + v1 c1) + (v0 c1 - v1 c0) u
        g.op([(v0, S(c0)), (v1, S(c1))], out[0])
        g.op([(v0, S(c1)), (scale(v1, -1), S(c0))], out[1])
    g.op([(Z[0], S(ONE))], Z3o[0])
    g.op([(scale(Z[1], -1), S(ONE))], Z3o[1])
    return g


def prog_psi2(src, dst):
    """psi^2(P) = (X cx2, Y cy2, Z), bls_curve.h g2_psi2"""
    g = Prog("psi2_%d%d" % (src, dst), bounds_with(src))
    X, Y, Z = (pair(t) for t in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    g.mulfp(X, S(PSI2_CX), out=X3o)
    g.mulfp(Y, S(PSI2_CY), out=Y3o)
    g.ident2(Z, Z3o)
    return g


def emit(progs):
    table, offsets = [], {}
    for g in progs:
        g.check()
        for t in bank(0) + bank(1) + bank(2) + bank(3) + bank(4) + bank(5):
            for s in t:
                if g.written.get(s, -1) >= 0:
                    assert g.bound[s] < PT_BOUND, (g.name, s, g.bound[s])
        offsets[g.name] = len(table)
        table.append(len(g.rounds))
        for rnd in g.rounds:
            T = max(len(l) for _, l in rnd)
            M = max(max(len(a[0]), len(b[0])) for _, l in rnd for a, b in l)
            table += [T, M]
            for lane in range(gm.LANES):
                out, lins = rnd[lane] if lane < len(rnd) else (DUMMY, [])
                table.append(out)
                for k in range(T):
                    for side in (0, 1):
                        items, K = (lins[k][side][0], lins[k][side][1]) if k < len(lins) else ([], 0)
                        for j in range(M):
                            if j < len(items):
                                s, c = items[j]
                                table += [s, c & 0xff]
                            else:
                                table += [ONE, 0]
                        table.append(K)
    nslots = max(g.next_temp for g in progs)
    L = ["// GENERATED by tools/gen_tcurve.py -- do not edit.",
         "// Team G2 point programs for the latency path (see the generator's docstring).",
         "#pragma once",
         "#define TCP_NSLOT %d" % nslots,
         "#define TCP_S_ONE %d" % ONE, "#define TCP_S_PSI_CX %d" % PSI_CX[0], "#define TCP_S_PSI_CY %d" % PSI_CY[0],
         "#define TCP_S_PSI2_CX %d" % PSI2_CX, "#define TCP_S_PSI2_CY %d" % PSI2_CY,
         "#define TCP_S_DUMMY %d" % DUMMY, "#define TCP_BANK(k) (%d + 6 * (k))" % BANK0]
    for name, off in offsets.items():
        L.append("#define TCP_%s %d" % (name.upper(), off))
    hh = set(HH_SLOTS.values())
    assert len(hh) == 1, hh  # every add program uses the same HH temporaries
    L.append("#define TCP_S_HH %d" % list(hh)[0][0])
    L.append("#define TCP_TABLE_BYTES %d" % len(table))
    L.append("#define TCP_TABLE_INIT {%s}" % ",".join(str(b) for b in table))
    return "\n".join(L) + "\n"


def main():
    progs = [prog_dbl(4, 5), prog_dbl(5, 4), prog_add(4, 0, 5), prog_add(5, 0, 4), prog_add(1, 2, 3),
             prog_psi(1, 2), prog_psi2(1, 2)]
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lodestar_amd", "csrc",
                       "bgv_tcurve_prog.h")
    open(out, "w").write(emit(progs))
    print("wrote", out, "slots", max(g.next_temp for g in progs), "bytes",
          sum(1 for _ in open(out).read().split(",")))


if __name__ == "__main__":
    main()
