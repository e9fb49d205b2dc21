"""The residue-number-system engine of the latency path's closing (bgv_rns.h, round 6): the
lane-level model in tools/gen_rns.py -- the exact arithmetic the device lanes run -- against
big integers mod p and the oracle's Fp12 products, and the committed constant header against
the generator (CPU; the device engine itself: tests/test_gpu_r06.py::test_rns_engine_probe and
every latency-path GPU test, whose closing k_final_fold runs it).  Reference: the final
exponentiation of blst's verifyMultipleAggregateSignatures (chain/bls/maybeBatch.ts:18-25)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_rns_model_against_big_integers_and_oracle():
    import gen_rns as g
    worst = g.check(n=60, seed=3)
    assert worst < g.KNEG


def test_rns_header_is_generated_from_the_model():
    import gen_rns as g
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "h.h")
        g.emit_header(out)
        want = open(out).read()
    got = open(os.path.join(ROOT, "lodestar_amd", "csrc", "bgv_rns_consts.h")).read()
    assert got == want, "bgv_rns_consts.h is stale: python tools/gen_rns.py"


def test_rns_reduction_edges():
    import gen_rns as g
    for L in g.LANES:
        for x in (0, 1, L["m"] - 1, L["m"], (1 << 64) - 1, (1 << 63) + 12345, L["m"] * ((1 << 35) + 7)):
            assert g.red64(x, L) == x % L["m"]
