"""Generates lodestar_amd/csrc/bgv_tcurve_prog.h: G2 point programs for a team of 16 lanes
(the latency path's cofactor clearing, r * sig and the subgroup check's [|x|]P, bgv_tcurve.h).

Same instruction model as tools/gen_tmiller.py (one Fp output per lane per round,
REDC(sum_k lin(A_k) lin(B_k)), bounds tracked per slot), over fixed point "banks" of six
Fp slots (X, Y, Z as Fp2 pairs).  The chains run in HOMOGENEOUS projective coordinates
(x = X/Z, y = Y/Z), whose formulas have lower degree than the Jacobian ones, so they need
fewer rounds (a round squares the degree at most):

  pdbl45 / pdbl54   doubling for y^2 = x^3 + b', b' = 4(1 + u):  U = 3b'Z^2,
                    X3 = 2XY (Y^2 - 3U), Y3 = Y^2 (Y^2 + 6U) - 3U^2, Z3 = 8 Y^2 (YZ)     2 rounds
                    (Jacobian dbl-2009-l: 3)
  padd405 / padd504 / padd123   addition (add-1998-cmo-2 regrouped): R1 the cross products
                    Y2Z1, Y1Z2, X2Z1, X1Z2, Z1Z2 (u, v linear in them); R2 u^2, v^2 and six
                    degree-4 products; R3 X3 = u^2 (v Z1Z2) - v^2 (v^2 + 2 v X1Z2),
                    Y3 = v^2 (3 u X1Z2 + uv - v Y1Z2) - u^2 (u Z1Z2), Z3 = v^2 (v Z1Z2)  3 rounds
                    (Jacobian add-2007-bl: 5)
  psi12 / psi2_12   g2_psi / g2_psi2: the same maps in either coordinates               1 round
  j2p12_45          Jacobian banks 1, 2 -> projective banks 4, 5: (XZ, Y, Z^3)         2 rounds
  iso12_45          the 3-isogeny of the SSWU points in banks 1, 2 (E2', Jacobian) into
                    projective banks 4, 5, both points side by side                     6 rounds
  p2j31             projective bank 3 -> Jacobian bank 1: (XZ, YZ^2, Z)                2 rounds

The schedules convert at their entry and exit, so every bank handed in or out is Jacobian,
as bls_curve.h's one-lane formulas use (same points, other representatives).  Additions
are the generic-case formulas; the driver checks v^2 != 0 and Z1Z2 != 0 (slots TCP_S_VV,
TCP_S_ZZ of the addition programs) and falls back to the complete one-lane formulas if
either ever is zero.

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


# the 3-isogeny's constants (RFC 9380 E.3, bls_hash.h iso_map_g2_jac), Fp2 pairs after the banks:
# x_num k1_0..3, x_den k2_0..1 (x^2 monic), y_num k3_0..3, y_den k4_0..2 (x^3 monic)
ISO0 = BANK0 + 6 * NBANK
ISO_XN = [(ISO0 + 2 * i, ISO0 + 2 * i + 1) for i in range(4)]
ISO_XD = [(ISO0 + 8 + 2 * i, ISO0 + 9 + 2 * i) for i in range(2)]
ISO_YN = [(ISO0 + 12 + 2 * i, ISO0 + 13 + 2 * i) for i in range(4)]
ISO_YD = [(ISO0 + 20 + 2 * i, ISO0 + 21 + 2 * i) for i in range(3)]
TEMP0 = ISO0 + 26
gm.TEMP0 = TEMP0  # Prog allocates temporaries from here
gm.ONE = ONE
gm.DUMMY = DUMMY

BOUND_IN = {ONE: 1, PSI_CX[0]: 1, PSI_CX[1]: 1, PSI_CY[0]: 1, PSI_CY[1]: 1, PSI2_CX: 1, PSI2_CY: 1}
for _t in ISO_XN + ISO_XD + ISO_YN + ISO_YD:
    BOUND_IN[_t[0]] = BOUND_IN[_t[1]] = 1
PT_BOUND = 2.0  # every bank value is weakly reduced (< 2p): checked on every program's outputs


def bounds_with(*banks):
    b = dict(BOUND_IN)
    for k in banks:
        for t in bank(k):
            for s in t:
                b[s] = PT_BOUND
    return b


def mul_b3(a):
    """3 b' a = 12 (1 + u) a as a pair of forms"""
    return (scale(add(a[0], scale(a[1], -1)), 12), scale(add(a[0], a[1]), 12))


def neg_prod(c, d):
    """-(c d) as extra product terms of mul2 (re, im)"""
    return ([(scale(c[0], -1), d[0]), (c[1], d[1])], [(scale(c[0], -1), d[1]), (scale(c[1], -1), d[0])])


def prog_pdbl(src, dst):
    g = Prog("pdbl%d%d" % (src, dst), bounds_with(src))
    X, Y, Z = (pair(t) for t in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    XY = g.mul2(X, Y)
    Y2 = g.sqr2(Y)
    YZ = g.mul2(Y, Z)
    U = g.mul2(Z, mul_b3(Z))
    g.new_round()
    g.mul2(lin2((2, XY)), lin2((1, Y2), (-3, U)), out=X3o)
    g.mul2(Y2, lin2((1, Y2), (6, U)), out=Y3o, extra=neg_prod(lin2((3, U)), U))
    g.mul2(lin2((8, Y2)), YZ, out=Z3o)
    return g


CHK_SLOTS = {}


def prog_padd(a, b, dst):
    g = Prog("padd%d%d%d" % (a, b, dst), bounds_with(a, b))
    X1, Y1, Z1 = (pair(t) for t in bank(a))
    X2, Y2, Z2 = (pair(t) for t in bank(b))
    X3o, Y3o, Z3o = bank(dst)
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
    CHK_SLOTS[g.name] = (list(vv[0])[0], list(ZZ[0])[0])
    return g


def pos_prod(c, d):
    """+(c d) as extra product terms of mul2 (re, im)"""
    return ([(c[0], d[0]), (scale(c[1], -1), d[1])], [(c[0], d[1]), (c[1], d[0])])


def cat(*ts):
    return (sum((list(t[0]) for t in ts), []), sum((list(t[1]) for t in ts), []))


def prog_iso(pairs, name):
    """The 3-isogeny E2' -> E2 of SSWU points (Jacobian, banks src) into projective banks dst,
    both maps' points side by side: with z2 = Z^2 and the maps homogenized (XNh = x_num z2^3,
    XDh = x_den z2^2, YNh = y_num z2^3, YDh = y_den z2^3), X' = XNh Z^3 YDh,
    Y' = Y YNh XDh z2, Z' = XDh z2 Z^3 YDh.  6 rounds, at most 16 instructions each."""
    g = Prog(name, bounds_with(*[s for s, _ in pairs]))
    k1 = [pair(t) for t in ISO_XN]
    k2 = [pair(t) for t in ISO_XD]
    k3 = [pair(t) for t in ISO_YN]
    k4 = [pair(t) for t in ISO_YD]
    st = {}
    for src, dst in pairs:
        X, Y, Z = (pair(t) for t in bank(src))
        st[src] = {"X": X, "Y": Y, "Z": Z, "z2": g.sqr2(Z), "X2": g.sqr2(X)}
    g.new_round()
    for src, _ in pairs:
        v = st[src]
        v["X3"] = g.mul2(v["X2"], v["X"])
        v["X2z2"] = g.mul2(v["X2"], v["z2"])
        v["Xz2"] = g.mul2(v["X"], v["z2"])
        v["z4"] = g.sqr2(v["z2"])
    g.new_round()
    for src, _ in pairs:
        v = st[src]
        v["Xz4"] = g.mul2(v["Xz2"], v["z2"])
        v["z6"] = g.mul2(v["z4"], v["z2"])
        v["XD"] = g.mul2(k2[1], v["Xz2"], extra=cat(pos_prod(k2[0], v["z4"]),
                                                   ([(v["X2"][0], S(ONE))], [(v["X2"][1], S(ONE))])))
        v["Z3"] = g.mul2(v["Z"], v["z2"])
    g.new_round()
    for src, _ in pairs:
        v = st[src]
        v["XN"] = g.mul2(k1[3], v["X3"], extra=cat(pos_prod(k1[2], v["X2z2"]), pos_prod(k1[1], v["Xz4"]),
                                                  pos_prod(k1[0], v["z6"])))
        v["YN"] = g.mul2(k3[3], v["X3"], extra=cat(pos_prod(k3[2], v["X2z2"]), pos_prod(k3[1], v["Xz4"]),
                                                  pos_prod(k3[0], v["z6"])))
        v["YD"] = g.mul2(k4[2], v["X2z2"], extra=cat(pos_prod(k4[1], v["Xz4"]), pos_prod(k4[0], v["z6"]),
                                                    ([(v["X3"][0], S(ONE))], [(v["X3"][1], S(ONE))])))
        v["XDz2"] = g.mul2(v["XD"], v["z2"])
    g.new_round()
    for src, _ in pairs:
        v = st[src]
        v["Z3YD"] = g.mul2(v["Z3"], v["YD"])
        v["W1"] = g.mul2(v["XDz2"], v["Y"])
    g.new_round()
    for src, dst in pairs:
        v = st[src]
        X3o, Y3o, Z3o = bank(dst)
        g.mul2(v["XN"], v["Z3YD"], out=X3o)
        g.mul2(v["W1"], v["YN"], out=Y3o)
        g.mul2(v["XDz2"], v["Z3YD"], out=Z3o)
    return g


def prog_j2p(pairs, name):
    """Jacobian (X, Y, Z) -> projective (X Z, Y, Z^3) for each (src, dst) bank pair"""
    g = Prog(name, bounds_with(*[s for s, _ in pairs]))
    zz = {}
    for src, dst in pairs:
        X, Y, Z = (pair(t) for t in bank(src))
        X3o, Y3o, _ = bank(dst)
        g.mul2(X, Z, out=X3o)
        g.ident2(Y, Y3o)
        zz[src] = g.sqr2(Z)
    g.new_round()
    for src, dst in pairs:
        Z = pair(bank(src)[2])
        g.mul2(Z, zz[src], out=bank(dst)[2])
    return g


def prog_p2j(src, dst):
    """projective (X, Y, Z) -> Jacobian (X Z, Y Z^2, Z)"""
    g = Prog("p2j%d%d" % (src, dst), bounds_with(src))
    X, Y, Z = (pair(t) for t in bank(src))
    X3o, Y3o, Z3o = bank(dst)
    g.mul2(X, Z, out=X3o)
    g.ident2(Z, Z3o)
    zz = g.sqr2(Z)
    g.new_round()
    g.mul2(Y, zz, out=Y3o)
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
         "#define TCP_S_DUMMY %d" % DUMMY, "#define TCP_BANK(k) (%d + 6 * (k))" % BANK0,
         "#define TCP_S_ISO %d  // x_num[4], x_den[2], y_num[4], y_den[3] (Fp2 pairs)" % ISO0]
    for name, off in offsets.items():
        L.append("#define TCP_%s %d" % (name.upper(), off))
    chk = set(CHK_SLOTS.values())
    assert len(chk) == 1, chk  # every addition program uses the same v^2 / Z1Z2 temporaries
    L.append("#define TCP_S_VV %d" % list(chk)[0][0])
    L.append("#define TCP_S_ZZ %d" % list(chk)[0][1])
    L.append("#define TCP_TABLE_BYTES %d" % len(table))
    L.append("#define TCP_TABLE_INIT {%s}" % ",".join(str(b) for b in table))
    return "\n".join(L) + "\n"


def main():
    progs = [prog_pdbl(4, 5), prog_pdbl(5, 4), prog_padd(4, 0, 5), prog_padd(5, 0, 4), prog_padd(1, 2, 3),
             prog_psi(1, 2), prog_psi2(1, 2), prog_j2p([(1, 4), (2, 5)], "j2p12_45"), prog_p2j(3, 1),
             prog_iso([(1, 4), (2, 5)], "iso12_45")]
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lodestar_amd", "csrc",
                       "bgv_tcurve_prog.h")
    open(out, "w").write(emit(progs))
    print("wrote", out, "slots", max(g.next_temp for g in progs), "bytes",
          sum(1 for _ in open(out).read().split(",")))


if __name__ == "__main__":
    main()
