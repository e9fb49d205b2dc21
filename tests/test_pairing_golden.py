"""Pairing values with injected randomizers (SURVEY 8(c) last row; VERDICT r03 "next" #2).

tests/golden/pairing.json (tools/gen_golden_r04.py, from the oracle pinned by
tests/test_oracle_kat.py) holds, per set of one call, the randomizer bgv_debug_prepare injects
(i-th nonzero splitmix64 word of the seed, r = lo + hi x^2 mod r), the oracle's Miller value and
the pairing value e(r_i pk_i, H(m_i)).  CPU tests here check the fixture against the oracle and
the bulk kernels' own math (host build: GLV r*pk, k_miller's miller_loop1, final_exp) against
it.  The GPU tests (test_gpu_pairing.py) compare the device's f_i on both paths.
Reference semantics: packages/beacon-node/src/chain/bls/maybeBatch.ts:18-25 (blst
verifyMultipleAggregateSignatures -> mul_n_aggregate per set, one final exponentiation).
"""
import json
import os

from oracle import bls12381 as o
from tests import hostsim as hs

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pairing.json")))


def f12_from_bytes(b):
    """576-byte tower-order serialisation -> the oracle's flat-w Fp12 tuple."""
    t = [int.from_bytes(b[48 * i:48 * i + 48], "big") for i in range(12)]
    flat = [None] * 6
    for k, j in enumerate((0, 2, 4, 1, 3, 5)):
        flat[j] = (t[2 * k], t[2 * k + 1])
    return tuple(flat)


def test_randomizer_derivation():
    import tools.gen_golden_r04 as g
    rs = g.randomizers(GOLD["seed"], len(GOLD["sets"]))
    for (w, r), s in zip(rs, GOLD["sets"]):
        assert "%016x" % w == s["word"] and int(s["r"], 16) == r
        assert 0 < r < o.R


def test_fixture_against_oracle():
    keys = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "keys.json")))
    sks = [int(v, 16) for v in keys["sk"]]
    for s in GOLD["sets"][:1] + GOLD["sets"][8:9]:
        pk = o.pubkey_aggregate([o.sk_to_pk(sks[k]) for k in s["pk_indices"]])
        h = o.hash_to_g2(bytes.fromhex(s["msg"]))
        m = f12_from_bytes(bytes.fromhex(s["miller"]))
        assert m == o.miller_loop(o.g1_mul(pk, int(s["r"], 16)), h)
        assert f12_from_bytes(bytes.fromhex(s["gt"])) == o.final_exp(m)


def test_bulk_kernel_math_matches_golden():
    """The bulk path's per-set pairing value computed by the kernels' own formulas (host
    build) equals the golden e(r pk, H(m)) -- cubed, since the kernels' final_exp computes the
    cube of the pairing (bls_pairing.h final_exp)."""
    keys = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "keys.json")))
    sks = [int(v, 16) for v in keys["sk"]]
    L = hs.lib()
    for s in GOLD["sets"][:2] + GOLD["sets"][9:10]:
        pk = o.pubkey_aggregate([o.sk_to_pk(sks[k]) for k in s["pk_indices"]])
        h = o.hash_to_g2(bytes.fromhex(s["msg"]))
        out = hs.buf(576)
        import ctypes
        L.hs_bulk_pair_value(out, hs.g1_b(pk), hs.g2_b(h), ctypes.c_uint64(int(s["word"], 16)))
        gt = f12_from_bytes(bytes.fromhex(s["gt"]))
        assert f12_from_bytes(out.raw) == o.f12_mul(o.f12_sqr(gt), gt)


def test_two_phase_miller_equals_single_pass():
    """k_lines + k_facc (P-free line records, then f over the records scaled by P) give the
    same pairing value as the single-pass miller_loop1m, for Jacobian P and Q with random Z
    (the bulk path's inputs are Jacobian).  Since round 6 the records' walk runs in projective
    coordinates (bls_pairing.h lz_pline_dbl_p / lz_pline_add_p): its lines are other
    representatives (Fp2 factors), so f agrees after the final exponentiation."""
    import ctypes
    import random
    L = hs.lib()
    rng = random.Random(4)
    for _ in range(3):
        pk = o.g1_mul(o.G1, rng.randrange(1, o.R))
        h = o.hash_to_g2(rng.randbytes(32))
        z1 = hs.fp_b(rng.randrange(1, o.P))
        z2 = hs.fp2_b((rng.randrange(o.P), rng.randrange(o.P)))
        a, b = hs.buf(576), hs.buf(576)
        L.hs_miller_two_phase(a, hs.g1_b(pk), hs.g2_b(h), z1, z2)
        L.hs_miller_one_pass(b, hs.g1_b(pk), hs.g2_b(h), z1, z2)
        fa, fb = hs.buf(576), hs.buf(576)
        L.hs_final_exp(fa, a.raw)
        L.hs_final_exp(fb, b.raw)
        assert fa.raw == fb.raw
        assert o.final_exp(f12_from_bytes(a.raw)) == o.pairing(pk, h) if _ == 0 else True
