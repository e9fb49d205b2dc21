"""CPU check of the wave-cooperative product algorithms (bgv_wfp.h wfp_mul3 / wfp_umul_l,
bgv_wround.h wr_instr) through the lane-level emulation in tools/emu_wfp.py: rotated operands,
the reduction as two more lane-parallel products, the carry passes and the ballot carry
lookahead against Montgomery products mod p.  The compiled kernels are checked against
fp_mul_body on the GPU (tools/ubench_wfp.hip, tools/ubench_wround.hip)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import emu_wfp as E  # noqa: E402


def test_wave_products_random():
    assert E.check(cases=9, seed=7) == 9


def test_wave_products_edges():
    rinv = pow(E.R, -1, E.P)
    for x, y in ((0, 5), (E.P - 1, E.P - 1), (2 * E.P - 1, 2 * E.P - 1), (1, E.R % E.P), (E.P, 3)):
        got = E.wfp_mul3(E.from_limbs(E.limbs(x)), E.from_limbs(E.limbs(y)))
        assert E.value(got) % E.P == x * y * rinv % E.P and E.value(got) < 2 * E.P
        u = E.wfp_umul(E.limbs(x), E.limbs(y))
        assert E.value(u) == E.value(got)
        # the same product through the signed round engine (one term, no combination)
        a = E.wr_lin(None, [(E.limbs(x), 1)], 0)
        b = E.wr_lin(None, [(E.limbs(y), 1)], 0)
        out = E.wr_reduce(E.wr_mac([0] * E.W, a, b))
        assert E.value(out) % E.P == x * y * rinv % E.P and all(0 <= v < 1 << E.LB for v in out[:E.NL])


def test_carry_lookahead_exact():
    # digits in [-1, 2^28 + 1] over the low lanes resolve to the same value, digits in range
    import random
    rng = random.Random(3)
    low = 0xFFFC000000000000
    for _ in range(200):
        d = [0] * E.W
        for L in range(50, 64):
            d[L] = rng.choice([-1, 0, E.MASK, 1 << E.LB, (1 << E.LB) + 1, rng.randrange(1 << E.LB)])
        want = sum(d[L] << (E.LB * (L - 50)) for L in range(50, 64))
        f, out = E.resolve(d, low)
        assert all(0 <= f[L] < 1 << E.LB for L in range(50, 64))
        assert sum(f[L] << (E.LB * (L - 50)) for L in range(50, 64)) + (out << (E.LB * 14)) == want
