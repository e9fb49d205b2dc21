"""Generate the golden fixtures under tests/golden/ with the CPU oracle.

    python tools/gen_golden.py

Every expected value comes from oracle/bls12381.py, which is itself pinned to
the reference's own known answers (tests/test_oracle_kat.py: the 100 interop
pubkeys of state-transition/test-cache/interop-pubkeys.json, the deposit-0
signature of beacon-node/test/e2e/interop/genesisState.test.ts:51-55, and the
RFC 9380 vectors).  The fixtures are data only (inputs and expected outputs).
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12381 as o  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
NKEYS = 128
FIXED_SCALARS_SEED = 0x5EED


def hx(b):
    return bytes(b).hex()


def sk_bytes(sk):
    return sk.to_bytes(32, "big")


def main():
    os.makedirs(OUT, exist_ok=True)
    # ---- keys: interop sk_i (state-transition/src/util/interop.ts:19-22) ----------
    sks = [o.interop_secret_key(i) for i in range(NKEYS)]
    pks = [o.sk_to_pk(sk) for sk in sks]
    ref = json.load(open(os.path.join(OUT, "interop-pubkeys.json")))
    for i in range(100):
        assert o.g1_compress(pks[i]).hex() == ref[i][2:], i
    # extra cache entry NKEYS = -pk_0, so that [0, NKEYS] aggregates to infinity
    neg0 = o.g1_neg(pks[0])
    keys = {
        "note": "interop secret keys sk_i (interop.ts:19-22) for i < %d; entry %d is -pk_0 (infinity aggregate)"
                % (NKEYS, NKEYS),
        "sk": [hx(sk_bytes(sk)) for sk in sks],
        "pk_compressed": [hx(o.g1_compress(p)) for p in pks] + [hx(o.g1_compress(neg0))],
        "pk_uncompressed": [hx(o.g1_serialize(p)) for p in pks] + [hx(o.g1_serialize(neg0))],
    }
    json.dump(keys, open(os.path.join(OUT, "keys.json"), "w"), indent=0)

    # ---- aggregates (PublicKey.aggregate + toBytes(uncompressed), utils.ts:5-16) -----
    agg_cases = [[0], [0, 1], [5, 5], list(range(NKEYS)), [3, 17, 99, 100, 127], [0, NKEYS], [7, 7, 7, 7]]
    all_pk = pks + [neg0]
    aggs = [{"indices": ix, "uncompressed": hx(o.g1_serialize(o.pubkey_aggregate([all_pk[i] for i in ix])))}
            for ix in agg_cases]
    json.dump({"note": "96-byte uncompressed aggregate pubkeys", "cases": aggs},
              open(os.path.join(OUT, "aggregates.json"), "w"), indent=0)

    # ---- hash_to_G2 (DST POP) ----------------------------------------------------
    msgs = [b"", b"abc", bytes(32), bytes([0xFF]) * 32, bytes(range(100)), b"a" * 255]
    msgs += [hashlib.sha256(b"lodestar-golden-%d" % i).digest() for i in range(58)]
    hashes = []
    for m in msgs:
        h = o.hash_to_g2(m)
        hashes.append({"msg": hx(m), "uncompressed": hx(o.g2_serialize(h)), "compressed": hx(o.g2_compress(h))})
    json.dump({"dst": o.DST_POP.decode(), "cases": hashes}, open(os.path.join(OUT, "hash_to_g2.json"), "w"),
              indent=0)

    # ---- signatures: sk_i * H(m) ---------------------------------------------------
    sig_cases = []
    for i in range(16):
        m = hashlib.sha256(b"lodestar-sign-%d" % i).digest()
        sig_cases.append({"key": i, "msg": hx(m), "sig": hx(o.g2_compress(o.sign(sks[i], m)))})
    json.dump({"cases": sig_cases}, open(os.path.join(OUT, "signatures.json"), "w"), indent=0)

    # ---- verdict vectors -----------------------------------------------------------
    def msg(i):
        return hashlib.sha256(b"lodestar-verdict-%d" % i).digest()

    def sig(k, m):
        return o.g2_compress(o.sign(sks[k], m))

    def single(k, m, s):
        return {"pk": [k], "msg": hx(m), "sig": hx(s)}

    good = [single(k, msg(k), sig(k, msg(k))) for k in range(8)]
    m_agg = msg(100)
    agg_sig = o.g2_compress(o.g2_add(o.g2_add(o.sign(sks[10], m_agg), o.sign(sks[11], m_agg)), o.sign(sks[12], m_agg)))
    agg_set = {"pk": [10, 11, 12], "msg": hx(m_agg), "sig": hx(agg_sig)}
    comp0 = bytes.fromhex(good[0]["sig"])
    # encodings that fail to decode
    no_flag = bytes([comp0[0] & 0x7F]) + comp0[1:]
    x_ge_p = bytes([0x80 | 0x1F]) + b"\xff" * 47 + comp0[48:]
    off_curve = None
    for k in range(1, 200):
        cand = bytearray(comp0)
        cand[95] ^= k
        try:
            o.g2_decompress(bytes(cand))
        except o.BlstError as e:
            if e.code == o.BLST_POINT_NOT_ON_CURVE:
                off_curve = bytes(cand)
                break
    assert off_curve is not None
    not_in_g2 = o.g2_compress(o.map_to_curve_g2((5, 7)))
    inf_sig = bytes([0xC0]) + bytes(95)

    jobs = []

    def job(name, sets, batchable=True):
        jobs.append({"name": name, "batchable": batchable, "sets": sets})

    job("valid_single", [good[0]])
    job("valid_three", good[1:4])
    job("valid_aggregate", [agg_set])
    job("wrong_msg", [single(4, msg(999), sig(4, msg(4)))])
    job("wrong_key", [single(5, msg(5), sig(6, msg(5)))])
    job("invalid_size_32", [{"pk": [0], "msg": hx(msg(0)), "sig": hx(bytes(32))}])
    job("bad_flag", [single(0, msg(0), no_flag)])
    job("x_ge_p", [single(0, msg(0), x_ge_p)])
    job("off_curve", [single(0, msg(0), off_curve)])
    job("not_in_g2", [single(0, msg(0), not_in_g2)])
    job("infinity_sig_single", [single(0, msg(0), inf_sig)])
    job("infinity_sig_in_pair", [good[5], single(0, msg(0), inf_sig)])
    job("empty_aggregate", [{"pk": [], "msg": hx(msg(0)), "sig": hx(comp0)}])
    job("empty_job", [])
    job("infinity_pk_single", [{"pk": [0, NKEYS], "msg": hx(msg(0)), "sig": hx(comp0)}])
    job("infinity_pk_pair", [good[6], {"pk": [0, NKEYS], "msg": hx(msg(0)), "sig": hx(comp0)}])
    job("wrong_then_malformed", [single(4, msg(999), sig(4, msg(4))), single(0, msg(0), no_flag)])
    job("valid_nonbatchable", [good[7], agg_set], batchable=False)
    job("wrong_nonbatchable", [good[2], single(4, msg(999), sig(4, msg(4)))], batchable=False)
    job("valid_after", good[5:8])

    import random
    rng = random.Random(FIXED_SCALARS_SEED)
    for jb in jobs:
        sets = []
        try:
            for s in jb["sets"]:
                if len(s["pk"]) == 0:
                    raise ValueError("EMPTY_AGGREGATE_ARRAY")
            for s in jb["sets"]:
                sets.append((o.pubkey_aggregate([all_pk[i] for i in s["pk"]]), bytes.fromhex(s["msg"]),
                             bytes.fromhex(s["sig"])))
            scalars = [rng.getrandbits(64) | 1 for _ in sets]
            jb["expect"] = 1 if o.verify_signature_sets_maybe_batch(sets, scalars) else 0
        except o.BlstError as e:
            jb["expect"] = -e.code
            jb["error"] = str(e)
        except ValueError as e:
            jb["expect"] = -20 if "EMPTY_AGGREGATE" in str(e) else -21
            jb["error"] = str(e)
        print(jb["name"], jb["expect"], flush=True)
    json.dump({"note": "expected per-job code: 1 valid, 0 invalid, -code error (include/blsgpu.h)",
               "jobs": jobs}, open(os.path.join(OUT, "verdicts.json"), "w"), indent=0)


if __name__ == "__main__":
    main()
