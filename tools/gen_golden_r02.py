"""Round-2 golden fixtures (tests/golden/r02.json) from the CPU oracle.

    python tools/gen_golden_r02.py

  pk_records   96-byte pubkey records (the SerializedSet.publicKey / bgv_set.pk_bytes
               format, multithread/worker.ts:110-116) decoded as blst's
               POINTonE1_Deserialize_Z: every flag combination, x >= p, off-curve,
               (0, 2); expected code, and for a decodable record the signature it
               verifies under (key 0's signature over a fixed root, or none)
  aggregates   PublicKey.aggregate(...).toBytes(uncompressed) (chain/bls/utils.ts:5-16) at
               1 / 2 / 16 / 128 / 512 keys, with repeated validators, partial sums that
               cancel to infinity, and a layout in which lanes l and l + 32 of the device
               tree hold equal partial sums (the doubling branch of the complete addition)

The oracle is pinned to the reference's own known answers (tests/test_oracle_kat.py).
Data only: inputs and expected outputs.
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12381 as o  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "r02.json")


def hx(b):
    return bytes(b).hex()


def code_of(fn, *a):
    try:
        return 0, fn(*a)
    except o.BlstError as e:
        return e.code, None


def main():
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    sks = [int(s, 16) for s in keys["sk"]]
    pks = [o.sk_to_pk(sk) for sk in sks]
    neg0 = o.g1_neg(pks[0])
    cache = pks + [neg0]  # the cache layout of tests/golden/keys.json (entry 128 = -pk_0)
    n = len(cache)

    # ---- 96-byte pubkey records ----------------------------------------------
    msg = hashlib.sha256(b"r02-pk-records").digest()
    sig0 = o.g2_compress(o.sign(sks[0], msg))
    good = bytearray(o.g1_serialize(pks[0]))
    comp = bytearray(o.g1_compress(pks[0]))
    recs = []

    def add(name, b):
        code, pt = code_of(o.g1_deserialize, bytes(b))
        recs.append({"name": name, "record": hx(b), "expect_code": code,
                     "infinity": code == 0 and pt is None,
                     "is_pk0": code == 0 and pt is not None and pt == pks[0]})

    add("uncompressed", good)
    b = bytearray(good); b[0] |= 0x20; add("sort_flag_without_compression", b)
    add("compressed_in_first_48", comp + bytes(48))
    add("compressed_in_first_48_trailing_junk", comp + bytes([0xAB]) * 48)
    add("infinity", bytes([0x40]) + bytes(95))
    b = bytearray([0x40]) + bytes(94) + bytes([1]); add("infinity_with_junk", b)
    b = bytearray([0x60]) + bytes(95); add("infinity_with_sort_flag", b)
    xp = o.P.to_bytes(48, "big"); add("x_equals_p", xp + good[48:])
    yp = o.P.to_bytes(48, "big"); add("y_equals_p", good[:48] + yp)
    b = bytearray(good); b[95] ^= 1; add("off_curve", b)
    add("x_zero_y_two", bytes(48) + (2).to_bytes(48, "big"))
    add("x_zero_y_minus_two", bytes(48) + (o.P - 2).to_bytes(48, "big"))
    add("compressed_x_zero", bytes([0x80]) + bytes(47) + bytes(48))

    # ---- pubkey aggregates -----------------------------------------------------
    def agg(ix):
        return hx(o.g1_serialize(o.pubkey_aggregate([cache[i] for i in ix])))

    cases = {
        "one": [5],
        "two": [5, 6],
        "sixteen": list(range(16)),
        "distinct_128": list(range(128)),
        "repeated_512": [(37 * k) % n for k in range(512)],
        # lane l and l + 32 of the 64-lane tree sum equal keys: the doubling branch
        "tree_lane_pairs_equal_512": [(k % 32 + 32 * (k // 64)) % n for k in range(512)],
        # every lane's partial sum is pk_0 + (-pk_0) = infinity; the total is infinity
        "tree_partials_infinity_128": [0] * 64 + [128] * 64,
        # an infinity aggregate of 2 keys and a 17-key set containing it
        "cancel_pair": [0, 128],
        "seventeen_with_cancel": [0, 128] + list(range(1, 16)),
        "same_key_64": [7] * 64,
    }
    aggs = [{"name": k, "indices": v, "uncompressed": agg(v)} for k, v in cases.items()]

    json.dump({"note": "round-2 fixtures from oracle/bls12381.py (tools/gen_golden_r02.py); cache = "
                       "tests/golden/keys.json pk_compressed (129 entries, entry 128 = -pk_0)",
               "pk_records": {"msg": hx(msg), "sig_by_key0": hx(sig0), "cases": recs},
               "aggregates": aggs}, open(OUT, "w"), indent=0)
    print("pk_records", [(r["name"], r["expect_code"]) for r in recs])
    print("aggregates", [(a["name"], len(a["indices"])) for a in aggs])


if __name__ == "__main__":
    main()
