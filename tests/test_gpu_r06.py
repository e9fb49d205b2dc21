"""GPU tests added in round 6.

Retry rounds of uniform groups just above the latency bound (advisor r05, high): a bulk call
whose first pass is uniform (nslots + ngroups > BGV_LATENCY_MAX, one Miller loop per group over
its pubkey sum) runs retry rounds with only a few test groups, so nslots + nrg can fall below
the bound.  The closing must still be k_final12 (it multiplies the tests' pubkey-sum pairs);
k_final_fold would multiply the uniform groups' unwritten per-slot f_i and reject valid jobs.
Every verdict must equal the job verified alone (chain/bls/multithread/worker.ts:76-98).
"""
import hashlib

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
NKEYS = 4096


def _sk(i):
    return (int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R).to_bytes(32, "big")


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd import native
    sks = [_sk(i) for i in range(NKEYS)]
    c = native.Context([0])
    c.keygen(b"".join(sks), cache_first=0, want_pubkeys=False)
    yield c, sks
    c.close()


@pytest.mark.parametrize("n", [16100, 16200, 16300])
def test_uniform_retry_just_above_latency_bound(ctx, n):
    from lodestar_amd import native
    c, sks = ctx
    committee = 128
    roots = [hashlib.sha256(b"r06-window-%d" % (i // committee)).digest() for i in range(n)]
    keys = [(i * 7) % NKEYS for i in range(n)]
    sigs = c.sign(b"".join(sks[k] for k in keys), b"".join(roots))
    sets = [native.SetSpec(roots[i], sigs[96 * i:96 * i + 96], pk_indices=[keys[i]]) for i in range(n)]
    want = [1] * n
    for i in (1, 64 * 3 + 17, 64 * 40 + 63, n - 2):  # one wrong key per failing group
        sets[i] = native.SetSpec(roots[i], sets[i].sig, pk_indices=[(keys[i] + 1) % NKEYS])
        want[i] = 0
    jobs = [([s], True) for s in sets]
    st = native.BgvStats()
    got = c.verify_jobs(jobs, native.MODE_WORKER, stats=st)
    assert got == want
    assert st.batch_retries >= 4


# ---------------------------------------------------------------------------------------
# Uniform groups pinned by value (VERDICT r05 "next" #2).  A group whose sets share one root
# takes ONE Miller loop over its pubkey sum, prod_i e(r_i pk_i, H) = e(sum_i r_i pk_i, H); its
# retry tests pair their own pubkey sums, and the weighted test weights slot k by k + 1.
# bgv_debug_uniform injects the randomizers (the i-th nonzero splitmix64 word of the seed,
# r = lo + hi x^2 mod r, as bgv_debug_prepare) and returns those Miller values; each is final-
# exponentiated here with the oracle's final exponentiation and compared with the oracle's
# pairing value.  With sig_i = sk_i H and pk_i = sk_i G1 every expected value is a power of
# gt = e(G1, H):  e(sum w_i r_i pk_i, H) = gt^a and e(-G1, sum w_i r_i sig_i) = gt^-a with
# a = sum w_i r_i sk_i (mod r).  Bit-exact integer work; reference:
# packages/beacon-node/src/chain/bls/maybeBatch.ts:18-25, multithread/worker.ts:76-98.
# ---------------------------------------------------------------------------------------
def test_uniform_group_values_pinned_to_oracle():
    import json
    import os
    from lodestar_amd import native
    from oracle import bls12381 as o
    from tests.test_pairing_golden import f12_from_bytes
    from tools.gen_golden_r04 import randomizers
    here = os.path.dirname(os.path.abspath(__file__))
    keys = json.load(open(os.path.join(here, "golden", "keys.json")))
    n = 40
    sks = [int(v, 16) for v in keys["sk"][:n]]
    c = native.Context([0])
    try:
        c.pubkeys_put(0, b"".join(bytes.fromhex(k) for k in keys["pk_compressed"][:n]), native.PK_COMPRESSED)
        msg = hashlib.sha256(b"r06-uniform-values").digest()
        sigs = c.sign(b"".join(sk.to_bytes(32, "big") for sk in sks), msg * n)
        sets = [native.SetSpec(msg, sigs[96 * i:96 * i + 96], pk_indices=[i]) for i in range(n)]
        seed = 0x5EED0006
        rs = [r for _, r in randomizers(seed, n)]
        wrong_slot = 23  # the weighted test names one slot; its weight is 24
        tests = [(sum(1 << k for k in range(n) if k & 1), False),          # a pattern test S_0
                 (sum(1 << k for k in range(n) if k & 4), False),          # S_2
                 ((1 << n) - 1, True),                                     # the weighted test
                 (((1 << n) - 1) & ~(1 << wrong_slot), True)]              # weighted, one slot dead
        first, vals = c.debug_uniform(sets, seed, tests)
    finally:
        c.close()
    gt = o.pairing(o.G1, o.hash_to_g2(msg))

    def expect(mask, weighted):
        a = sum(((k + 1) if weighted else 1) * rs[k] * sks[k] for k in range(n) if (mask >> k) & 1) % o.R
        return o.f12_pow(gt, a)

    assert o.final_exp(f12_from_bytes(first)) == expect((1 << n) - 1, False)
    for (mask, weighted), (pk576, sig576) in zip(tests, vals):
        e = expect(mask, weighted)
        assert o.final_exp(f12_from_bytes(pk576)) == e, (hex(mask), weighted, "pubkey-sum pair")
        assert o.final_exp(f12_from_bytes(sig576)) == o.f12_inv(e), (hex(mask), weighted, "signature pair")


# ---------------------------------------------------------------------------------------
# The residue-number-system Fp12 engine of k_final_fold (bgv_rns.h): its tm_pow_x chain, its
# fp_t conversions in and out, and the eight-part engine it replaced, each checked against the
# oracle on the same random Fp12 value (tools/gpu/rns_probe.py over tools/bin/ubench_rns, built
# by __graft_entry__.build()); the probe also times both engines.
# ---------------------------------------------------------------------------------------
def test_rns_engine_probe():
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tools", "bin", "ubench_rns")
    assert os.path.exists(exe), "tools/bin/ubench_rns missing: run __graft_entry__.build()"
    res = subprocess.run([sys.executable, os.path.join(root, "tools", "gpu", "rns_probe.py"), "2", "11"],
                         capture_output=True, text=True, timeout=180)
    assert res.returncode == 0, res.stdout + res.stderr
    verdict = json.loads(res.stdout.strip().splitlines()[-1])
    assert verdict["rns_chain_ok"] and verdict["rns_from_fp_ok"] and verdict["rns_to_fp_ok"] and verdict["part8_chain_ok"]
    assert verdict["rns_output_bound_p"] < 16


# ---------------------------------------------------------------------------------------
# Root-aligned layout (round 6, bgv_api.cpp call_submit): roots with >= 32 one-set jobs start
# device groups of their own, the smaller roots share mixed groups after them; a pattern unit
# whose every index bit failed both ways goes to singles.  Roots of 100, 40, 33, 32, 31, 5 and 1
# jobs interleaved in call order, wrong keys inside the large roots, a mixed region whose jobs
# are all invalid (every pattern bit fails), and a valid singleton: every verdict must equal the
# job verified alone (multithread/worker.ts:76-98).
# ---------------------------------------------------------------------------------------
def test_root_aligned_layout_verdicts(ctx):
    import random
    from lodestar_amd import native
    c, sks = ctx
    rnd = random.Random(0xA11C)
    sizes = [100, 40, 1, 33, 5, 32, 31, 1, 1, 100] + [1] * 40
    roots, order = [], []
    for r, n in enumerate(sizes):
        roots.append(hashlib.sha256(b"r06-layout-%d" % r).digest())
        order += [r] * n
    rnd.shuffle(order)  # roots recur after one another: the grouped layout
    n = len(order)
    msgs = [roots[r] for r in order]
    keys = [(i * 13) % NKEYS for i in range(n)]
    sigs = c.sign(b"".join(sks[k] for k in keys), b"".join(msgs))
    sets = [native.SetSpec(msgs[i], sigs[96 * i:96 * i + 96], pk_indices=[keys[i]]) for i in range(n)]
    want = [1] * n
    big = [i for i in range(n) if sizes[order[i]] >= 32]
    for i in rnd.sample(big, 6):  # wrong keys inside the aligned roots
        sets[i] = native.SetSpec(msgs[i], sets[i].sig, pk_indices=[(keys[i] + 1) % NKEYS])
        want[i] = 0
    small = [i for i in range(n) if sizes[order[i]] == 1]
    for i in small[:-1]:  # the mixed region all invalid but one
        sets[i] = native.SetSpec(msgs[i], sets[i].sig, pk_indices=[(keys[i] + 3) % NKEYS])
        want[i] = 0
    # pad the call past the bulk/uniform thresholds with valid distinct-root sets (call order)
    extra = 16384  # bulk batch (nslots + ngroups > BGV_LATENCY_MAX): uniform groups and weighted tests
    emsgs = [hashlib.sha256(b"r06-layout-extra-%d" % i).digest() for i in range(extra)]
    ekeys = [(7 * i + 1) % NKEYS for i in range(extra)]
    esigs = c.sign(b"".join(sks[k] for k in ekeys), b"".join(emsgs))
    sets += [native.SetSpec(emsgs[i], esigs[96 * i:96 * i + 96], pk_indices=[ekeys[i]]) for i in range(extra)]
    want += [1] * extra
    jobs = [([s], True) for s in sets]
    st = native.BgvStats()
    assert c.verify_jobs(jobs, native.MODE_WORKER, stats=st) == want
    assert st.batch_retries >= 1
