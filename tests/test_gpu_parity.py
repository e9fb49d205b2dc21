"""GPU parity tests: libblsgpu.so (HIP, gfx950) against the oracle's golden vectors.

Every expected value is a committed fixture (tests/golden/, made by
tools/gen_golden.py from oracle/bls12381.py, which tests/test_oracle_kat.py
pins to the reference's interop pubkeys, deposit-0 signature and RFC 9380).
Integer work: every comparison is bit-exact.
"""
import asyncio
import hashlib
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return json.load(open(os.path.join(GOLD, name)))


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd import native
    c = native.Context()
    keys = load("keys.json")
    c.pubkeys_put(0, b"".join(bytes.fromhex(k) for k in keys["pk_compressed"]), native.PK_COMPRESSED)
    yield c
    c.close()


def test_pubkey_cache_and_aggregate(ctx):
    keys = load("keys.json")
    assert ctx.pubkeys_count() == len(keys["pk_compressed"])
    for case in load("aggregates.json")["cases"]:
        assert ctx.aggregate_pubkeys(case["indices"]).hex() == case["uncompressed"], case["indices"]


def test_pubkeys_uncompressed_roundtrip(ctx):
    from lodestar_amd import native
    keys = load("keys.json")
    c2 = native.Context()
    c2.pubkeys_put(0, b"".join(bytes.fromhex(k) for k in keys["pk_uncompressed"][:8]), native.PK_UNCOMPRESSED)
    for i in range(8):
        assert c2.aggregate_pubkeys([i]).hex() == keys["pk_uncompressed"][i]
    c2.close()


def test_hash_to_g2(ctx):
    cases = load("hash_to_g2.json")["cases"]
    outs = ctx.hash_to_g2([bytes.fromhex(c["msg"]) for c in cases])
    for c, got in zip(cases, outs):
        assert got.hex() == c["uncompressed"], c["msg"]


def test_keygen_matches_interop_pubkeys(ctx):
    keys = load("keys.json")
    sks = b"".join(bytes.fromhex(s) for s in keys["sk"])
    pks = ctx.keygen(sks)
    for i in range(len(keys["sk"])):
        assert pks[48 * i:48 * i + 48].hex() == keys["pk_compressed"][i], i


def test_sign(ctx):
    keys = load("keys.json")
    cases = load("signatures.json")["cases"]
    sks = b"".join(bytes.fromhex(keys["sk"][c["key"]]) for c in cases)
    msgs = b"".join(bytes.fromhex(c["msg"]) for c in cases)
    sigs = ctx.sign(sks, msgs)
    for i, c in enumerate(cases):
        assert sigs[96 * i:96 * i + 96].hex() == c["sig"], i


def _jobs_from_golden():
    from lodestar_amd import native
    jobs, expect, names = [], [], []
    for jb in load("verdicts.json")["jobs"]:
        sets = [native.SetSpec(bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]), pk_indices=s["pk"])
                for s in jb["sets"]]
        jobs.append((sets, jb["batchable"]))
        expect.append(jb["expect"])
        names.append(jb["name"])
    return jobs, expect, names


@pytest.mark.parametrize("mode", [0, 1])
def test_verdict_vectors(ctx, mode):
    from lodestar_amd import native
    jobs, expect, names = _jobs_from_golden()
    stats = native.BgvStats()
    got = ctx.verify_jobs(jobs, mode, stats)
    assert dict(zip(names, got)) == dict(zip(names, expect))
    if mode == 0:
        assert stats.batch_retries >= 1  # the shared group holding wrong_msg/wrong_key failed


def test_verdict_vectors_one_by_one(ctx):
    jobs, expect, names = _jobs_from_golden()
    for j, e, n in zip(jobs, expect, names):
        assert ctx.verify_jobs([j], 0) == [e], n


def test_uncached_pubkey_bytes(ctx):
    """SerializedSet path: 96-byte uncompressed pubkeys uploaded with the call (worker.ts:110-116)."""
    from lodestar_amd import native
    keys = load("keys.json")
    sigs = load("signatures.json")["cases"]
    sets = [native.SetSpec(bytes.fromhex(c["msg"]), bytes.fromhex(c["sig"]),
                           pk_bytes=[bytes.fromhex(keys["pk_uncompressed"][c["key"]])]) for c in sigs[:4]]
    assert ctx.verify_jobs([(sets, True)]) == [1]
    bad = bytearray.fromhex(keys["pk_uncompressed"][0])
    bad[95] ^= 1  # off the curve
    sets[1] = native.SetSpec(sets[1].msg, sets[1].sig, pk_bytes=[bytes(bad)])
    assert ctx.verify_jobs([(sets, True)]) == [-2]


def _mk_batch(ctx, n, seed, corrupt_frac=0.0, nkeys=128):
    """n single sets over the golden keys, device-signed; returns (sets, expected_codes)."""
    from lodestar_amd import native
    keys = load("keys.json")
    rng = random.Random(seed)
    ks = [rng.randrange(nkeys) for _ in range(n)]
    msgs = [hashlib.sha256(b"batch-%d-%d" % (seed, i)).digest() for i in range(n)]
    sigs = ctx.sign(b"".join(bytes.fromhex(keys["sk"][k]) for k in ks), b"".join(msgs))
    sigs = [sigs[96 * i:96 * i + 96] for i in range(n)]
    expect = [1] * n
    bad = rng.sample(range(n), int(round(n * corrupt_frac)))
    for j, i in enumerate(bad):
        kind = j % 3
        if kind == 0:  # wrong message -> false
            msgs[i] = hashlib.sha256(b"other" + msgs[i]).digest()
            expect[i] = 0
        elif kind == 1:  # signature by another key -> false
            ks[i] = (ks[i] + 1) % nkeys
            expect[i] = 0
        else:  # flip the compression flag -> BLST_BAD_ENCODING
            sigs[i] = bytes([sigs[i][0] & 0x7F]) + sigs[i][1:]
            expect[i] = -1
    sets = [native.SetSpec(msgs[i], sigs[i], pk_indices=[ks[i]]) for i in range(n)]
    return sets, expect


def test_gossip_batch_with_retry(ctx):
    """Config-4 shape at test size: 512 batchable one-set jobs, 1% corrupted."""
    from lodestar_amd import native
    sets, expect = _mk_batch(ctx, 512, 0x8192, 0.01)
    stats = native.BgvStats()
    got = ctx.verify_jobs([([s], True) for s in sets], 0, stats)
    assert got == expect
    assert stats.batch_retries >= 1
    # one call holding every set -> the single job is invalid/error like the reference
    got1 = ctx.verify_jobs([(sets, False)], 0)
    assert got1 == [-1]


def test_block_import_shape(ctx):
    """Config-3 shape: randao + aggregate attestations + sync aggregate + proposer, one
    non-batchable call.  Aggregates use the same message for all members."""
    from lodestar_amd import native
    keys = load("keys.json")
    sk = [bytes.fromhex(s) for s in keys["sk"]]
    m = hashlib.sha256(b"attestation-data").digest()
    members = list(range(0, 128, 3))
    sigs = ctx.sign(b"".join(sk[i] for i in members), m * len(members))
    import oracle.bls12381 as o
    agg = None
    for i in range(len(members)):
        agg = o.g2_add(agg, o.signature_from_bytes(sigs[96 * i:96 * i + 96]))
    agg_sig = o.g2_compress(agg)
    single_m = hashlib.sha256(b"randao").digest()
    single_sig = ctx.sign(sk[3], single_m)
    sets = [native.SetSpec(single_m, single_sig, pk_indices=[3]),
            native.SetSpec(m, agg_sig, pk_indices=members)]
    assert ctx.verify_jobs([(sets, False)], 0) == [1]
    sets2 = [sets[0], native.SetSpec(m, agg_sig, pk_indices=members[:-1])]
    assert ctx.verify_jobs([(sets2, False)], 0) == [0]


def test_blsgpuverifier_e2e():
    """beacon-node/test/e2e/chain/bls/multithread.test.ts:60-103 on BlsGpuVerifier:
    sk_i = bytes32(fill i+1), msg_i = bytes32(fill i+1); concurrent sync / batchable calls,
    and one invalid (32-byte) signature rejecting with BLST_INVALID_SIZE while the
    others resolve true."""
    from lodestar_amd import native
    from lodestar_amd.verifier import BlsGpuVerifier, ISignatureSet, SignatureSetType, VerifySignatureOpts, QueueError

    async def run():
        c = native.Context()
        sks = b"".join(bytes([i + 1]) * 32 for i in range(3))
        c.keygen(sks, cache_first=0, want_pubkeys=False)
        msgs = [bytes([i + 1]) * 32 for i in range(3)]
        sigs = c.sign(sks, b"".join(msgs))
        sets = [ISignatureSet(SignatureSetType.single, msgs[i], sigs[96 * i:96 * i + 96], pubkey=i)
                for i in range(3)]
        v = BlsGpuVerifier(c)
        for opts in (None, VerifySignatureOpts(batchable=True), VerifySignatureOpts(verify_on_main_thread=True)):
            res = await asyncio.gather(*[v.verify_signature_sets(sets, opts) for _ in range(8)])
            assert res == [True] * 8
        bad = [ISignatureSet(SignatureSetType.single, msgs[0], bytes(32), pubkey=0)]
        tasks = [v.verify_signature_sets(sets, VerifySignatureOpts(batchable=True)) for _ in range(8)]
        tasks.append(v.verify_signature_sets(bad, VerifySignatureOpts(batchable=True)))
        res = await asyncio.gather(*tasks, return_exceptions=True)
        assert res[:8] == [True] * 8
        assert isinstance(res[8], native.BlsGpuError) and "BLST_INVALID_SIZE" in str(res[8])
        await v.close()
        with pytest.raises(QueueError):
            await v.verify_signature_sets(sets)
        c.close()

    asyncio.run(run())


def test_pubkeys_validate_golden(ctx):
    """Deposit-time key validation (processDeposit.ts:64) against tests/golden/next.json."""
    cases = load("next.json")["pubkeys"]
    codes, recs = ctx.pubkeys_validate([bytes.fromhex(c["pk"]) for c in cases])
    assert codes == [-c["expect"] for c in cases]
    keys = load("keys.json")
    for i in range(8):  # valid keys come back as the uncompressed cache record
        assert recs[i].hex() == keys["pk_uncompressed"][i]


def test_aggregate_signatures_golden(ctx):
    """Op-pool Signature.aggregate over validated signatures, golden aggregates."""
    cases = load("next.json")["aggregates"]
    got = ctx.aggregate_signatures([[bytes.fromhex(s) for s in c["sigs"]] for c in cases])
    for c, (code, agg) in zip(cases, got):
        assert code == -c["expect"], c
        if c["expect"] == 0:
            assert agg.hex() == c["aggregate"]


def test_deposits_verify_golden(ctx):
    cases = load("next.json")["deposits"]
    got = ctx.deposits_verify([bytes.fromhex(c["pk"]) for c in cases], [bytes.fromhex(c["msg"]) for c in cases],
                              [bytes.fromhex(c["sig"]) for c in cases])
    assert got == [c["expect"] for c in cases]


def test_light_client_is_valid_bls_aggregate(ctx):
    """light-client/src/validation.ts:152-176 isValidBlsAggregate on BlsGpuVerifier: a sync
    aggregate over golden keys (96-B uncompressed pubkeys, as the light client holds PublicKey
    objects) verifies; a wrong root is false; an empty key list and an undecodable signature raise
    with the dependency's codes; the infinity aggregate (k and -k) verifies false."""
    from lodestar_amd import native
    from lodestar_amd.verifier import BlsGpuVerifier
    from oracle import bls12381 as o  # checker only
    keys = load("keys.json")
    n = min(16, len(keys["sk"]))
    sks = [int(k, 16) for k in keys["sk"][:n]]
    pks = [bytes.fromhex(k) for k in keys["pk_uncompressed"][:n]]
    root = hashlib.sha256(b"lc-sync-aggregate").digest()
    agg_sk = sum(sks) % o.R
    sig = ctx.sign(agg_sk.to_bytes(32, "big"), root)

    async def run():
        v = BlsGpuVerifier(ctx)
        assert await v.is_valid_bls_aggregate(pks, root, sig) is True
        assert await v.is_valid_bls_aggregate(pks, hashlib.sha256(b"other").digest(), sig) is False
        assert await v.is_valid_bls_aggregate(pks[:-1], root, sig) is False
        with pytest.raises(native.BlsGpuError) as e:
            await v.is_valid_bls_aggregate([], root, sig)
        assert e.value.code == native.BGV_E_EMPTY_AGGREGATE
        with pytest.raises(native.BlsGpuError) as e:
            await v.is_valid_bls_aggregate(pks, root, bytes([sig[0] & 0x7F]) + sig[1:])
        assert e.value.code == native.BLST_BAD_ENCODING
        neg = o.g1_serialize(o.sk_to_pk(o.R - sks[0]))
        assert await v.is_valid_bls_aggregate([pks[0], neg], root, sig) is False
        await v.close()

    asyncio.run(run())
