"""Generates lodestar_amd/csrc/bgv_tg1_prog.h: G1 point programs for the latency path's
r_i * pk_i (bgv_tg1.h), in the round model of tools/gen_tmiller.py (one Fp output per lane
per round, REDC(sum_k lin(A_k) lin(B_k)), bounds tracked per slot).

G1 banks hold three Fp slots (X, Y, Z).  The chains run in homogeneous projective
coordinates on y^2 = x^3 + 4 (3b = 12), with the same regrouped formulas as the G2 programs
(tools/gen_tcurve.py), on Fp values instead of Fp2 pairs:

  pdbl45 / pdbl54          2 rounds (4 + 3 instructions)
  padd405 / padd504 / padd123   3 rounds (5 + 8 + 3 instructions)
  endo12                   (beta X, -Y, Z) = [x^2] on G1 (bls_curve.h jac_endo_x2)   1 round
  j2p1_4                   Jacobian bank 1 -> projective bank 4: (XZ, Y, Z^3)        2 rounds
  p2j31                    projective bank 3 -> Jacobian bank 1: (XZ, YZ^2, Z)       2 rounds

    python tools/gen_tg1.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_tmiller as gm  # noqa: E402
from gen_tmiller import Prog, S, add, scale  # noqa: E402

ONE = 0
BETA = 1
DUMMY = 2
NBANK = 10
BANK0 = 3


def bank(k):
    b = BANK0 + 3 * k
    return (b, b + 1, b + 2)


TEMP0 = BANK0 + 3 * NBANK
gm.TEMP0 = TEMP0
gm.ONE = ONE
gm.DUMMY = DUMMY

BOUND_IN = {ONE: 1, BETA: 1}
PT_BOUND = 2.0


def bounds_with(*banks):
    b = dict(BOUND_IN)
    for k in banks:
        for s in bank(k):
            b[s] = PT_BOUND
    return b


def lin(*terms):
    return add(*[scale(f, c) for c, f in terms])


def prog_pdbl(src, dst):
    g = Prog("pdbl%d%d" % (src, dst), bounds_with(src))
    X, Y, Z = (S(s) for s in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    XY = g.op([(X, Y)])
    Y2 = g.op([(Y, Y)])
    YZ = g.op([(Y, Z)])
    U = g.op([(Z, scale(Z, 12))])  # 3 b Z^2
    g.new_round()
    g.op([(scale(XY, 2), lin((1, Y2), (-3, U)))], X3o)
    g.op([(Y2, lin((1, Y2), (6, U))), (scale(U, -3), U)], Y3o)
    g.op([(scale(Y2, 8), YZ)], Z3o)
    return g


CHK_SLOTS = {}


def prog_padd(a, b, dst):
    g = Prog("padd%d%d%d" % (a, b, dst), bounds_with(a, b))
    X1, Y1, Z1 = (S(s) for s in bank(a))
    X2, Y2, Z2 = (S(s) for s in bank(b))
    X3o, Y3o, Z3o = bank(dst)
    A1 = g.op([(Y2, Z1)])
    A2 = g.op([(Y1, Z2)])
    B1 = g.op([(X2, Z1)])
    B2 = g.op([(X1, Z2)])
    ZZ = g.op([(Z1, Z2)])
    g.new_round()
    u = lin((1, A1), (-1, A2))
    v = lin((1, B1), (-1, B2))
    uu = g.op([(u, u)])
    vv = g.op([(v, v)])
    vZZ = g.op([(v, ZZ)])
    vB2 = g.op([(v, B2)])
    uB2 = g.op([(u, B2)])
    uZZ = g.op([(u, ZZ)])
    uv = g.op([(u, v)])
    vA2 = g.op([(v, A2)])
    g.new_round()
    g.op([(uu, vZZ), (scale(vv, -1), lin((1, vv), (2, vB2)))], X3o)
    g.op([(vv, lin((3, uB2), (1, uv), (-1, vA2))), (scale(uu, -1), uZZ)], Y3o)
    g.op([(vv, vZZ)], Z3o)
    CHK_SLOTS[g.name] = (list(vv)[0], list(ZZ)[0])
    return g


def prog_endo(src, dst):
    g = Prog("endo%d%d" % (src, dst), bounds_with(src))
    X, Y, Z = (S(s) for s in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    g.op([(X, S(BETA))], X3o)
    g.op([(scale(Y, -1), S(ONE))], Y3o)
    g.op([(Z, S(ONE))], Z3o)
    return g


def prog_j2p(src, dst):
    g = Prog("j2p%d_%d" % (src, dst), bounds_with(src))
    X, Y, Z = (S(s) for s in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    g.op([(X, Z)], X3o)
    g.op([(Y, S(ONE))], Y3o)
    zz = g.op([(Z, Z)])
    g.new_round()
    g.op([(Z, zz)], Z3o)
    return g


def prog_p2j(src, dst):
    g = Prog("p2j%d%d" % (src, dst), bounds_with(src))
    X, Y, Z = (S(s) for s in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    g.op([(X, Z)], X3o)
    g.op([(Z, S(ONE))], Z3o)
    zz = g.op([(Z, Z)])
    g.new_round()
    g.op([(Y, zz)], Y3o)
    return g


def emit(progs):
    table, offsets = [], {}
    for g in progs:
        g.check()
        for k in range(NBANK):
            for s in bank(k):
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
                                assert -128 <= c < 128
                                table += [s, c & 0xff]
                            else:
                                table += [ONE, 0]
                        table.append(K)
    nslots = max(g.next_temp for g in progs)
    chk = set(CHK_SLOTS.values())
    assert len(chk) == 1, chk
    L = ["// GENERATED by tools/gen_tg1.py -- do not edit.",
         "// G1 point programs for the latency path's r * pk (see the generator's docstring).",
         "#pragma once",
         "#define TG1_NSLOT %d" % nslots,
         "#define TG1_S_ONE %d" % ONE, "#define TG1_S_BETA %d" % BETA, "#define TG1_S_DUMMY %d" % DUMMY,
         "#define TG1_BANK(k) (%d + 3 * (k))" % BANK0,
         "#define TG1_S_VV %d" % list(chk)[0][0], "#define TG1_S_ZZ %d" % list(chk)[0][1]]
    for name, off in offsets.items():
        L.append("#define TG1_%s %d" % (name.upper(), off))
    L.append("#define TG1_TABLE_BYTES %d" % len(table))
    L.append("#define TG1_TABLE_INIT {%s}" % ",".join(str(b) for b in table))
    L.append("// rounds: %s" % ", ".join("%s %d" % (g.name, len(g.rounds)) for g in progs))
    return "\n".join(L) + "\n"


def main():
    progs = [prog_pdbl(4, 5), prog_pdbl(5, 4), prog_padd(4, 0, 5), prog_padd(5, 0, 4), prog_padd(1, 2, 3),
             prog_endo(1, 2), prog_j2p(1, 4), prog_p2j(3, 1)]
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lodestar_amd", "csrc",
                       "bgv_tg1_prog.h")
    open(out, "w").write(emit(progs))
    print("wrote", out, "slots", max(g.next_temp for g in progs))


if __name__ == "__main__":
    main()
