"""Pins the CPU oracle (oracle/bls12381.py) to the reference's own known-answer data.

* interop-pubkeys.json: copied verbatim from
  /root/reference/packages/state-transition/test-cache/interop-pubkeys.json
  (100 compressed G1 pubkeys for sk_i of state-transition/src/util/interop.ts:19-22).
* deposit-0 signature: beacon-node/test/e2e/interop/genesisState.test.ts:51-55
  (minimal preset, GENESIS_FORK_VERSION 0x00000001; signing root built as in
  beacon-node/src/node/utils/interop/deposits.ts:23-31).
* RFC 9380 published vectors (expand_message_xmd J.10.1, hash_to_curve J.10.1 msg="").
"""
import hashlib
import json
import os

from oracle import bls12381 as o

H = lambda b: hashlib.sha256(b).digest()  # noqa: E731


def test_interop_pubkeys(golden_dir):
    pks = json.load(open(os.path.join(golden_dir, "interop-pubkeys.json")))
    assert len(pks) == 100
    for i in range(100):  # every one of the reference's 100 known answers
        assert o.g1_compress(o.sk_to_pk(o.interop_secret_key(i))).hex() == pks[i][2:]
        # decompress round trip
        pt = o.g1_decompress(bytes.fromhex(pks[i][2:]))
        assert o.g1_compress(pt).hex() == pks[i][2:]


def deposit0_signing_root(fork_version=b"\x00\x00\x00\x01"):
    sk = o.interop_secret_key(0)
    pk = o.g1_compress(o.sk_to_pk(sk))
    wc = b"\x00" + H(pk)[1:]
    amount = (32000000000).to_bytes(8, "little") + bytes(24)
    dm_root = H(H(H(pk[:32] + pk[32:] + bytes(16)) + wc) + H(amount + bytes(32)))
    domain = b"\x03\x00\x00\x00" + H(fork_version + bytes(60))[:28]
    return sk, pk, wc, H(dm_root + domain)


DEPOSIT0_SIG = (
    "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
    "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446"
)


def test_deposit0_signature_kat():
    sk, pk, wc, root = deposit0_signing_root()
    assert wc.hex() == "00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b"
    assert o.g2_compress(o.sign(sk, root)).hex() == DEPOSIT0_SIG
    # and it verifies through the pairing
    sig = o.signature_from_bytes(bytes.fromhex(DEPOSIT0_SIG))
    assert o.core_verify(o.g1_decompress(pk), root, sig)
    assert not o.core_verify(o.g1_decompress(pk), bytes(32), sig)


def test_rfc9380_vectors():
    assert (o.expand_message_xmd(b"", b"QUUX-V01-CS02-with-expander-SHA256-128", 0x20).hex()
            == "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235")
    h = o.hash_to_g2(b"", b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_")
    assert h[0] == (0x0141EBFBDCA40EB85B87142E130AB689C673CF60F1A3E98D69335266F30D9B8D4AC44C1038E9DCDD5393FAF5C41FB78A,
                    0x05CB8437535E20ECFFAEF7752BADDF98034139C38452458BAEEFAB379BA13DFF5BF5DD71B72418717047F5B0F37DA03D)


def test_algebra():
    assert o.g1_on_curve(o.G1) and o.g2_on_curve(o.G2)
    assert o.g2_mul(o.G2, o.R) is None
    q = o.g2_add(o.map_to_curve_g2((5, 7)), o.map_to_curve_g2((9, 11)))
    assert o.clear_cofactor_g2(q) == o.g2_mul(q, o.H_EFF_G2)
    e = o.pairing(o.G1, o.G2)
    assert o.pairing(o.g1_mul(o.G1, 3), o.g2_mul(o.G2, 5)) == o.f12_pow(e, 15)


def test_chunkify_reference_cases():
    # beacon-node/test/unit/chain/bls/utils.test.ts
    want = [[[0]], [[0, 1]], [[0, 1, 2]], [[0, 1, 2, 3]], [[0, 1, 2, 3, 4]],
            [[0, 1, 2], [3, 4, 5]], [[0, 1, 2, 3], [4, 5, 6]], [[0, 1, 2, 3], [4, 5, 6, 7]]]
    for i, w in enumerate(want):
        assert o.chunkify_maximize_chunk_size(list(range(i + 1)), 3) == w


def test_batch_semantics():
    sks = [int.from_bytes(bytes([i + 1]) * 32, "big") for i in range(3)]  # multithread.test.ts:25-38
    msgs = [bytes([i + 1]) * 32 for i in range(3)]
    pks = [o.sk_to_pk(sk) for sk in sks]
    sigs = [o.g2_compress(o.sign(sk, m)) for sk, m in zip(sks, msgs)]
    sets = list(zip(pks, msgs, sigs))
    assert o.verify_signature_sets_maybe_batch(sets, [3, 5, 7])
    bad = [(pks[0], msgs[1], sigs[0])] + sets[1:]
    assert not o.verify_signature_sets_maybe_batch(bad, [3, 5, 7])
    try:
        o.verify_signature_sets_maybe_batch([(pks[0], msgs[0], bytes(32))])
        assert False
    except o.BlstError as e:
        assert "BLST_INVALID_SIZE" in str(e)


def test_next_rows_oracle(golden_dir):
    """Oracle restatements for SURVEY 8(f): every reference interop pubkey
    (state-transition/test-cache/interop-pubkeys.json) passes deposit validation;
    the committed next.json fixtures agree with the oracle."""
    import json
    import os
    ref = json.load(open(os.path.join(golden_dir, "interop-pubkeys.json")))
    for h in ref[:16]:
        assert o.pubkey_validate(bytes.fromhex(h[2:])) == 0
    nxt = json.load(open(os.path.join(golden_dir, "next.json")))
    for c in nxt["pubkeys"]:
        assert o.pubkey_validate(bytes.fromhex(c["pk"])) == c["expect"]
    for c in nxt["aggregates"][:5]:
        code, agg = o.signatures_aggregate([bytes.fromhex(s) for s in c["sigs"]])
        assert code == c["expect"] and (agg.hex() if agg else None) == c["aggregate"]


def test_r02_fixtures_oracle(golden_dir):
    """tests/golden/r02.json (tools/gen_golden_r02.py) agrees with the pinned oracle:
    96-byte pubkey records decode (or reject) as blst's POINTonE1_Deserialize_Z, and the
    aggregates are PublicKey.aggregate(...).toBytes(uncompressed) of the cached keys."""
    fx = json.load(open(os.path.join(golden_dir, "r02.json")))
    keys = json.load(open(os.path.join(golden_dir, "keys.json")))
    cache = [o.g1_decompress(bytes.fromhex(k)) for k in keys["pk_compressed"]]
    for c in fx["pk_records"]["cases"]:
        try:
            pt, code = o.g1_deserialize(bytes.fromhex(c["record"])), 0
        except o.BlstError as e:
            pt, code = None, e.code
        assert code == c["expect_code"], c["name"]
        assert (code == 0 and pt is None) == c["infinity"], c["name"]
    for a in fx["aggregates"]:
        agg = o.pubkey_aggregate([cache[i] for i in a["indices"]])
        assert o.g1_serialize(agg).hex() == a["uncompressed"], a["name"]
