"""CPU unit tests of the kernel math (lodestar_amd/csrc/bls_*.h compiled for the
host as tests/native/libhostsim.so) against the oracle, oracle/bls12381.py.

Every device formula — Montgomery CIOS, Fp2 sqrt, line functions, Miller
loop, final exponentiation, SSWU/iso/cofactor, ZCash decoding — is checked
here bit-for-bit before it ever runs on an MI355X.
"""
import hashlib
import random

import pytest

from oracle import bls12381 as o
from tests import hostsim as hs

rnd = random.Random(0xB15)
P = o.P


def rfp():
    return rnd.randrange(P)


def rfp2():
    return (rfp(), rfp())


@pytest.fixture(scope="module", params=["wide", "classic"])
def L(request):
    return hs.lib(request.param)


def test_fp_ops(L):
    for _ in range(50):
        a, b = rfp(), rfp()
        r = hs.buf(48)
        L.hs_fp_mul(r, hs.fp_b(a), hs.fp_b(b))
        assert hs.b_fp(r.raw) == a * b % P
        L.hs_fp_add(r, hs.fp_b(a), hs.fp_b(b))
        assert hs.b_fp(r.raw) == (a + b) % P
        L.hs_fp_sub(r, hs.fp_b(a), hs.fp_b(b))
        assert hs.b_fp(r.raw) == (a - b) % P
        L.hs_fp_neg(r, hs.fp_b(a))
        assert hs.b_fp(r.raw) == (-a) % P
        L.hs_fp_half(r, hs.fp_b(a))
        assert hs.b_fp(r.raw) * 2 % P == a
    for a in (0, 1, P - 1, 2**380, P // 2):
        r = hs.buf(48)
        L.hs_fp_mul(r, hs.fp_b(a), hs.fp_b(P - 1))
        assert hs.b_fp(r.raw) == a * (P - 1) % P
        L.hs_fp_neg(r, hs.fp_b(a))
        assert hs.b_fp(r.raw) == (-a) % P
    a = rfp()
    r = hs.buf(48)
    L.hs_fp_inv(r, hs.fp_b(a))
    assert hs.b_fp(r.raw) * a % P == 1


def test_fp_sqrt(L):
    for _ in range(8):
        a = rfp()
        r = hs.buf(48)
        ok = L.hs_fp_sqrt(r, hs.fp_b(a))
        assert bool(ok) == o.fp_is_square(a)
        if ok:
            assert hs.b_fp(r.raw) ** 2 % P == a


def test_fp2_ops(L):
    for _ in range(20):
        a, b = rfp2(), rfp2()
        r = hs.buf(96)
        L.hs_fp2_mul(r, hs.fp2_b(a), hs.fp2_b(b))
        assert hs.b_fp2(r.raw) == o.f2_mul(a, b)
        L.hs_fp2_sqr(r, hs.fp2_b(a))
        assert hs.b_fp2(r.raw) == o.f2_sqr(a)
    a = rfp2()
    r = hs.buf(96)
    L.hs_fp2_inv(r, hs.fp2_b(a))
    assert o.f2_mul(hs.b_fp2(r.raw), a) == (1, 0)


def test_fp2_sqrt(L):
    cases = [rfp2() for _ in range(8)] + [(rfp(), 0), (0, rfp()), (0, 0), (4, 0), (P - 4, 0)]
    cases += [o.f2_sqr(rfp2()) for _ in range(4)]
    for a in cases:
        r = hs.buf(96)
        ok = L.hs_fp2_sqrt(r, hs.fp2_b(a))
        assert bool(ok) == o.f2_is_square(a), a
        if ok:
            assert o.f2_sqr(hs.b_fp2(r.raw)) == (a[0] % P, a[1] % P)


def rand_f12():
    return tuple(rfp2() for _ in range(6))


def f12_tower_bytes(f):
    return hs.fp12_b_tower(o.f12_to_tower_list(f))


def test_fp12_ops(L):
    a, b = rand_f12(), rand_f12()
    r = hs.buf(576)
    L.hs_fp12_mul(r, f12_tower_bytes(a), f12_tower_bytes(b))
    assert hs.b_fp12_tower(r.raw) == o.f12_to_tower_list(o.f12_mul(a, b))
    L.hs_fp12_sqr(r, f12_tower_bytes(a))
    assert hs.b_fp12_tower(r.raw) == o.f12_to_tower_list(o.f12_sqr(a))
    L.hs_fp12_frob(r, f12_tower_bytes(a))
    assert hs.b_fp12_tower(r.raw) == o.f12_to_tower_list(o.f12_frob(a))
    L.hs_fp12_frob2(r, f12_tower_bytes(a))
    assert hs.b_fp12_tower(r.raw) == o.f12_to_tower_list(o.f12_frob(o.f12_frob(a)))
    L.hs_fp12_inv(r, f12_tower_bytes(a))
    assert hs.b_fp12_tower(r.raw) == o.f12_to_tower_list(o.f12_inv_fast(a))
    # sparse line product: l0 at w^0, l1 at w^2, l3 at w^3
    l0, l1, l3 = rfp2(), rfp2(), rfp2()
    line = (l0, o.F2_ZERO, l1, l3, o.F2_ZERO, o.F2_ZERO)
    L.hs_fp12_mul_line(r, f12_tower_bytes(a), hs.fp2_b(l0), hs.fp2_b(l1), hs.fp2_b(l3))
    assert hs.b_fp12_tower(r.raw) == o.f12_to_tower_list(o.f12_mul(a, line))


def test_cyclotomic_sqr(L):
    a = rand_f12()
    # project into the cyclotomic subgroup with the easy part
    t = o.f12_mul(o.f12_conj(a), o.f12_inv_fast(a))
    t = o.f12_mul(o.f12_frob(o.f12_frob(t)), t)
    r = hs.buf(576)
    L.hs_fp12_cyc_sqr(r, f12_tower_bytes(t))
    assert hs.b_fp12_tower(r.raw) == o.f12_to_tower_list(o.f12_sqr(t))


def g2_rand_in_group():
    return o.g2_mul(o.G2, rnd.randrange(1, o.R))


def test_g2_arith(L):
    q1, q2 = g2_rand_in_group(), g2_rand_in_group()
    r = hs.buf(192)
    assert L.hs_g2_add(r, hs.g2_b(q1), hs.g2_b(q2))
    assert hs.b_g2(r.raw) == o.g2_add(q1, q2)
    assert L.hs_g2_add(r, hs.g2_b(q1), hs.g2_b(q1))  # equal inputs -> doubling
    assert hs.b_g2(r.raw) == o.g2_add(q1, q1)
    assert not L.hs_g2_add(r, hs.g2_b(q1), hs.g2_b(o.g2_neg(q1)))  # -> infinity
    assert L.hs_g2_dbl(r, hs.g2_b(q1))
    assert hs.b_g2(r.raw) == o.g2_add(q1, q1)
    for k in (1, 2, 3, 5, 0xFFFFFFFFFFFFFFFF, rnd.getrandbits(64)):
        assert L.hs_g2_mul_u64(r, hs.g2_b(q1), hs.ctypes.c_uint64(k))
        assert hs.b_g2(r.raw) == o.g2_mul(q1, k)
    assert L.hs_g2_psi(r, hs.g2_b(q1))
    assert hs.b_g2(r.raw) == o.g2_psi(q1)


def test_g2_subgroup_and_cofactor(L):
    q = g2_rand_in_group()
    assert L.hs_g2_in_subgroup(hs.g2_b(q)) == 1
    nq = o.map_to_curve_g2(rfp2())  # on E2, (almost surely) not in G2
    assert o.g2_on_curve(nq)
    assert L.hs_g2_on_curve(hs.g2_b(nq)) == 1
    assert L.hs_g2_in_subgroup(hs.g2_b(nq)) == 0
    r = hs.buf(192)
    assert L.hs_g2_clear_cofactor(r, hs.g2_b(nq))
    cc = hs.b_g2(r.raw)
    assert cc == o.clear_cofactor_g2(nq)
    assert L.hs_g2_in_subgroup(hs.g2_b(cc)) == 1


def test_g1_arith(L):
    p1 = o.g1_mul(o.G1, rnd.randrange(1, o.R))
    p2 = o.g1_mul(o.G1, rnd.randrange(1, o.R))
    r = hs.buf(96)
    assert L.hs_g1_add(r, hs.g1_b(p1), hs.g1_b(p2))
    assert hs.b_g1(r.raw) == o.g1_add(p1, p2)
    k = rnd.getrandbits(64)
    assert L.hs_g1_mul_u64(r, hs.g1_b(p1), hs.ctypes.c_uint64(k))
    assert hs.b_g1(r.raw) == o.g1_mul(p1, k)


def test_glv_randomizer_scalar_mult(L):
    """jac_mul_glv: r P with r = lo32(k) + hi32(k) x^2 mod the group order (the batch
    randomizers, bls_curve.h), on G1 (endomorphism (beta x, -y)) and G2 (psi^2), equal to
    the oracle's [r]P, including a = 0, b = 0, all-ones halves and small values."""
    x2 = (o.X * o.X) % o.R
    q = g2_rand_in_group()
    p = o.g1_mul(o.G1, rnd.randrange(1, o.R))
    r2, r1 = hs.buf(192), hs.buf(96)
    ks = [1, 2, 1 << 32, (1 << 32) | 1, 0xFFFFFFFF, 0xFFFFFFFF00000000, 0xFFFFFFFFFFFFFFFF, 7 << 32]
    ks += [rnd.getrandbits(64) | 1 for _ in range(3)]
    for k in ks:
        r = ((k & 0xFFFFFFFF) + (k >> 32) * x2) % o.R
        assert L.hs_g2_mul_glv(r2, hs.g2_b(q), hs.ctypes.c_uint64(k))
        assert hs.b_g2(r2.raw) == o.g2_mul(q, r), hex(k)
        assert L.hs_g1_mul_glv(r1, hs.g1_b(p), hs.ctypes.c_uint64(k))
        assert hs.b_g1(r1.raw) == o.g1_mul(p, r), hex(k)


def test_hash_to_g2_pieces(L):
    msg = bytes(range(32))
    r = hs.buf(192)
    L.hs_hash_to_field(r, msg, 32)
    u0, u1 = o.hash_to_field_fp2(msg, o.DST_POP)
    assert hs.b_g2(r.raw) == (u0, u1)
    for u in (u0, u1, rfp2(), rfp2(), rfp2()):
        L.hs_sswu(r, hs.fp2_b(u))
        assert hs.b_g2(r.raw) == o.sswu_g2(u)
    pt = o.sswu_g2(u0)
    assert L.hs_iso_map(r, hs.g2_b(pt))
    assert hs.b_g2(r.raw) == o.iso_map_g2(pt)


def test_sswu_iso_jacobian_without_inversion(L):
    """sswu_g2_jac + iso_map_g2_jac (the kernels' maps: Jacobian, no inversion, the square
    root of the ratio gx1 = U/V through the norm method) equal the oracle's affine maps, for
    random u (both square / non-square branches), u = 0 (the exceptional x1 = B/(ZA)) and
    the hash_to_field outputs."""
    r = hs.buf(192)
    msg = bytes(range(32))
    us = list(o.hash_to_field_fp2(msg, o.DST_POP)) + [rfp2() for _ in range(12)] + [(0, 0), (1, 0), (0, 1)]
    branches = set()
    for u in us:
        assert L.hs_sswu_iso_jac(r, hs.fp2_b(u))
        assert hs.b_g2(r.raw) == o.iso_map_g2(o.sswu_g2(u)), u
        branches.add(o.f2_is_square(o.f2_add(o.f2_mul(o.f2_add(o.f2_sqr(_x1(u)), o.SSWU_A), _x1(u)), o.SSWU_B)))
    assert branches == {True, False}


def _x1(u):
    """RFC 9380 6.6.2 x1 of the simplified SWU map (the oracle's formulas)"""
    tv1 = o.f2_mul(o.SSWU_Z, o.f2_sqr(u))
    tv2 = o.f2_add(o.f2_sqr(tv1), tv1)
    if o.f2_is_zero(tv2):
        return o.f2_mul(o.SSWU_B, o.f2_inv(o.f2_mul(o.SSWU_Z, o.SSWU_A)))
    return o.f2_mul(o.f2_mul(o.f2_neg(o.SSWU_B), o.f2_inv(o.SSWU_A)), o.f2_add((1, 0), o.f2_inv(tv2)))


@pytest.mark.parametrize("msg", [b"", b"abc", bytes(32), bytes([7]) * 32, bytes(range(100))])
def test_hash_to_g2(L, msg):
    aff, comp = hs.buf(192), hs.buf(96)
    assert L.hs_hash_to_g2(aff, comp, msg, len(msg))
    h = o.hash_to_g2(msg)
    assert hs.b_g2(aff.raw) == h
    assert comp.raw == o.g2_compress(h)


def test_g2_decompress(L):
    q = g2_rand_in_group()
    comp = o.g2_compress(q)
    r = hs.buf(192)
    assert L.hs_g2_decompress(r, comp) == 0
    assert hs.b_g2(r.raw) == q
    c = hs.buf(96)
    L.hs_g2_compress(c, hs.g2_b(q))
    assert c.raw == comp
    # infinity
    assert L.hs_g2_decompress(r, bytes([0xC0]) + bytes(95)) == 100
    # bad flags / non-canonical / off-curve
    assert L.hs_g2_decompress(r, bytes([0x00]) + comp[1:]) == o.BLST_BAD_ENCODING
    assert L.hs_g2_decompress(r, bytes([0xC0]) + bytes(94) + b"\x01") == o.BLST_BAD_ENCODING
    big = bytearray(comp)
    big[0] = 0x80 | 0x1F
    big[1:48] = b"\xff" * 47
    assert L.hs_g2_decompress(r, bytes(big)) == o.BLST_BAD_ENCODING
    # find an x that is not on the curve
    for k in range(1, 50):
        cand = bytearray(comp)
        cand[95] ^= k
        try:
            o.g2_decompress(bytes(cand))
        except o.BlstError as e:
            assert L.hs_g2_decompress(r, bytes(cand)) == e.code
            break


def test_g1_decompress(L, golden_dir):
    import json
    import os
    pks = json.load(open(os.path.join(golden_dir, "interop-pubkeys.json")))
    r = hs.buf(96)
    for h in pks[:5]:
        b = bytes.fromhex(h[2:])
        assert L.hs_g1_decompress(r, b) == 0
        pt = hs.b_g1(r.raw)
        assert pt == o.g1_decompress(b)
        s = hs.buf(96)
        L.hs_g1_serialize(s, hs.g1_b(pt))
        assert s.raw == o.g1_serialize(pt)


def test_pairing(L):
    p = o.g1_mul(o.G1, rnd.randrange(1, o.R))
    q = g2_rand_in_group()
    ml = hs.buf(576)
    L.hs_miller_loop(ml, hs.g1_b(p), hs.g2_b(q))
    fe = hs.buf(576)
    L.hs_final_exp(fe, ml.raw)
    want = o.f12_pow(o.pairing(p, q), 3)  # device final exp computes e(P,Q)^3
    assert hs.b_fp12_tower(fe.raw) == o.f12_to_tower_list(want)


def test_miller_loop1_and_team_loop(L):
    """The per-set one-pair loop (k_miller) and the team loop of the group closing
    (k_final, emulated lane by lane) both equal the oracle's Miller loop up to factors the
    final exponentiation kills; Q goes in Jacobian with Z != 1.  The team loop and the
    one-lane loop compute the same lines, so they agree exactly."""
    p = o.g1_mul(o.G1, rnd.randrange(1, o.R))
    q = g2_rand_in_group()
    ref, m1, tm = hs.buf(576), hs.buf(576), hs.buf(576)
    L.hs_miller_loop(ref, hs.g1_b(p), hs.g2_b(q))
    L.hs_miller_loop1(m1, hs.g1_b(p), hs.g2_b(q))
    L.hs_team_miller(tm, hs.g1_b(p), hs.g2_b(q))
    assert tm.raw == m1.raw
    fe = lambda m: (lambda out: (L.hs_final_exp(out, m), out.raw)[1])(hs.buf(576))
    assert fe(m1.raw) == fe(ref.raw)


def test_table_driven_team_miller_loop(L):
    """The latency path's team Miller loop (bgv_tmiller.h: generated twist-point rounds in
    projective coordinates, tools/gen_tmiller.py, and the coefficient-parallel Fp12
    accumulator), emulated lane by lane, gives miller_loop1's pairing value (its lines differ
    by Fp2 factors only) for random pairs and for -G1 with a random Q, and a different Q a
    different value."""
    fe = lambda m: (lambda out: (L.hs_final_exp(out, m), out.raw)[1])(hs.buf(576))
    for k in range(3):
        p = o.g1_mul(o.G1, rnd.randrange(1, o.R)) if k else o.g1_neg(o.G1)
        q = g2_rand_in_group()
        m1, tm = hs.buf(576), hs.buf(576)
        L.hs_miller_loop1(m1, hs.g1_b(p), hs.g2_b(q))
        want = fe(m1.raw)
        L.hs_tmiller(tm, hs.g1_b(p), hs.g2_b(q))
        assert tm.raw != m1.raw and fe(tm.raw) == want
        L.hs_tmiller_wide(tm, hs.g1_b(p), hs.g2_b(q))  # k_miller_wide: four-part instructions
        assert fe(tm.raw) == want
        L.hs_tmiller(tm, hs.g1_b(p), hs.g2_b(g2_rand_in_group()))
        assert fe(tm.raw) != want


def test_team_g1_schedule(L):
    """r * pk through the latency path's G1 point programs (bgv_tg1.h, projective, emulated
    lane by lane, plain and as four-part instructions) equals jac_mul_glv as a point, for
    random keys and randomizer words (full, a single low digit, a 40-bit word, a high half only)."""
    import ctypes
    for wide in (0, 1):
        L.hs_set_wide_rounds(wide)
        try:
            for scalar in (rnd.getrandbits(64) | 1, 1, rnd.getrandbits(40) | 1, 1 << 45, (1 << 64) - 1):
                p = o.g1_mul(o.G1, rnd.randrange(1, o.R))
                assert L.hs_tg1_check(hs.g1_b(p), ctypes.c_uint64(scalar)) == 1, (wide, scalar)
        finally:
            L.hs_set_wide_rounds(0)


def test_team_g2_schedules(L):
    """The latency path's team cofactor clearing and r * sig (bgv_tcurve.h, generated point
    programs, emulated lane by lane) equal g2_clear_cofactor and jac_mul_glv as points, for
    random messages and randomizer words (including zero top digits and a word of 1)."""
    import ctypes
    for wide in (0, 1):  # 1: the rounds as four-part instructions (k_prep_wide)
        L.hs_set_wide_rounds(wide)
        try:
            for k, m in enumerate((b"a", b"tcurve", b"x" * 7)):
                msg = hashlib.sha256(m).digest()
                scalar = (rnd.getrandbits(64) | 1) if k == 0 else (1 if k == 1 else rnd.getrandbits(40) | 1)
                bad = ctypes.c_int(7)
                assert L.hs_tcurve_check(msg, ctypes.c_uint64(scalar), ctypes.byref(bad)) == 1
                assert bad.value == 0
        finally:
            L.hs_set_wide_rounds(0)


def test_team_mul_line(L):
    """Coefficient-parallel product with a sparse line equals the tower formula."""
    for _ in range(4):
        f = rf12()
        l0, l1, l3 = (hs.fp2_b((rfp(), rfp())) for _ in range(3))
        want, got = hs.buf(576), hs.buf(576)
        L.hs_fp12_mul_line(want, f, l0, l1, l3)
        L.hs_team_mul_line(got, f, l0, l1, l3)
        assert got.raw == want.raw
        L.hs_team_mul_line_wide(got, f, l0, l1, l3)  # four parts per coefficient (k_miller_wide)
        assert got.raw == want.raw
        L.hs_team_mul_line_wide8(got, f, l0, l1, l3)  # eight parts per coefficient
        assert got.raw == want.raw


def test_verify_one_blst_equation(L):
    """k_prep (r pk, r sig) + k_miller e(r pk, H) + the group's team loop e(-G1, r sig)
    + the team final check for one set: valid -> 1, a signature by another key -> 0."""
    sk = o.interop_secret_key(5)
    pk = o.sk_to_pk(sk)
    msg = bytes(range(32))
    h = o.hash_to_g2(msg)
    sig = o.sign(sk, msg)
    r = rnd.getrandbits(64) | 1
    assert L.hs_verify_one(hs.g1_b(pk), hs.g2_b(h), hs.g2_b(sig), hs.ctypes.c_uint64(r)) == 1
    other = o.sign(o.interop_secret_key(6), msg)
    assert L.hs_verify_one(hs.g1_b(pk), hs.g2_b(h), hs.g2_b(other), hs.ctypes.c_uint64(r)) == 0


def rf12():
    return hs.fp12_b_tower([rfp() for _ in range(12)])


def test_team_fp12_ops(L):
    """Coefficient-parallel Fp12 product / Frobenius maps (bls_team.h) against the
    tower formulas, including operands with limbs at the 2p bound."""
    two_p_minus_1 = hs.fp12_b_tower([P - 1] * 12)
    for a, b in [(rf12(), rf12()) for _ in range(6)] + [(two_p_minus_1, two_p_minus_1)]:
        want, got = hs.buf(576), hs.buf(576)
        L.hs_fp12_mul(want, a, b)
        L.hs_team_mul(got, a, b)
        assert got.raw == want.raw
        L.hs_team_mul_wide(got, a, b)  # four parts per coefficient (latency-path closing)
        assert got.raw == want.raw
        L.hs_team_mul_wide8(got, a, b)  # eight parts per coefficient (k_final_fold)
        assert got.raw == want.raw
        L.hs_fp12_sqr(want, a)
        L.hs_team_sqr(got, a)  # 7-product team squaring
        assert got.raw == want.raw
        L.hs_team_sqr_wide(got, a)
        assert got.raw == want.raw
        L.hs_team_sqr_wide8(got, a)
        assert got.raw == want.raw
        L.hs_team_sqr_wide8_lean(got, a)  # operand recipes per lane (k_final_fold)
        assert got.raw == want.raw
        assert L.hs_team_sqr8_lean_diff(a) == 0  # the same 96 parts, limb for limb
        assert L.hs_team_sqr4_lean_diff(a) == 0  # the four-part form (k_miller_wide)
        for tf, ref in ((L.hs_team_frob, L.hs_fp12_frob), (L.hs_team_frob2, L.hs_fp12_frob2)):
            tf(got, a)
            ref(want, a)
            assert got.raw == want.raw
        L.hs_team_conj(got, a)
        assert hs.b_fp12_tower(got.raw) == hs.b_fp12_tower(a)[:6] + [(-x) % P for x in hs.b_fp12_tower(a)[6:]]


def test_team_final_exp_check(L):
    """The inversion-free quotient check agrees with final_exp(f) == 1: random f
    (not 1) and f = e(P, Q) e(-P, Q) Miller values (1), and a perturbed product."""
    for _ in range(2):
        f = rf12()
        assert L.hs_final_is_one(f) == 0
        assert L.hs_team_final_is_one(f) == 0
        assert L.hs_team_final_is_one_wide(f) == 0
        assert L.hs_team_final_is_one_wide8(f) == 0
        assert L.hs_team_final_is_one_wide8_lean(f) == 0
    p = o.g1_mul(o.G1, rnd.randrange(1, o.R))
    q = g2_rand_in_group()
    # e(P, Q) e(-P, Q) == 1 and e(P, Q) e(-P, Q2) != 1 (Miller values multiplied)
    m, a, b = hs.buf(576), hs.buf(576), hs.buf(576)
    L.hs_miller_loop(a, hs.g1_b(p), hs.g2_b(q))
    L.hs_miller_loop(b, hs.g1_b(o.g1_neg(p)), hs.g2_b(q))
    L.hs_fp12_mul(m, a.raw, b.raw)
    assert L.hs_final_is_one(m.raw) == 1
    assert L.hs_team_final_is_one(m.raw) == 1
    assert L.hs_team_final_is_one_wide(m.raw) == 1
    assert L.hs_team_final_is_one_wide8(m.raw) == 1
    assert L.hs_team_final_is_one_wide8_lean(m.raw) == 1
    q2 = g2_rand_in_group()
    L.hs_miller_loop(b, hs.g1_b(o.g1_neg(p)), hs.g2_b(q2))
    L.hs_fp12_mul(m, a.raw, b.raw)
    assert L.hs_final_is_one(m.raw) == 0
    assert L.hs_team_final_is_one(m.raw) == 0
    assert L.hs_team_final_is_one_wide(m.raw) == 0
    assert L.hs_team_final_is_one_wide8(m.raw) == 0
    assert L.hs_team_final_is_one_wide8_lean(m.raw) == 0


def test_wide_fp2_products_equal_classic():
    """bls_wide.h's deferred-reduction Fp2 product, Fp2-by-Fp product and squaring (the bulk
    kernels' tower, blst mul_mont_384x style) against the fully reduced Karatsuba, mod p: random
    operands at five bound pairs (limbs up to 2^29, values up to 40 p) and the
    extreme ones (every limb at its bound, zero).  The host build also checks every lazy bound."""
    for variant in ("wide", "classic"):
        assert hs.lib(variant).hs_wide_check(400, 0xB15 + len(variant)) == 0
