"""Golden fixtures for the SURVEY §8(f) rows built after the verify path:
deposit-time pubkey validation, op-pool signature aggregation and deposit
verification.  Expected values come from oracle/bls12381.py (pubkey_validate,
signatures_aggregate, deposit_valid); written to tests/golden/next.json.

    python tools/gen_golden_next.py
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12381 as o  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "next.json")


def g1_off_group():
    """A point on E(Fp) outside G1 (cofactor not cleared), compressed."""
    x = 1
    while True:
        y = o.fp_sqrt((x * x * x + o.B1) % o.P)
        if y is not None and not o.g1_in_group((x, y)):
            return o.g1_compress((x, y))
        x += 1


def g1_off_curve():
    x = 1
    while o.fp_sqrt((x * x * x + o.B1) % o.P) is not None:
        x += 1
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80
    return bytes(b)


def g2_off_group():
    k = 1
    while True:
        x = (k, 1)
        y = o.f2_sqrt(o.f2_add(o.f2_mul(o.f2_sqr(x), x), o.B2))
        if y is not None and not o.g2_in_group((x, y)):
            return o.g2_compress((x, y))
        k += 1


def main():
    sks = [o.interop_secret_key(i) for i in range(8)]
    pks = [o.sk_to_pk(sk) for sk in sks]
    bad_flag = bytearray(o.g1_compress(pks[0]))
    bad_flag[0] &= 0x7F
    big_x = bytearray((o.P + 1).to_bytes(48, "big"))
    big_x[0] |= 0x80
    inf_bad = bytearray([0xC0] + [0] * 47)
    inf_bad[47] = 1
    pk_cases = [o.g1_compress(p) for p in pks] + [
        bytes([0xC0]) + bytes(47), bytes(bad_flag), bytes(big_x), g1_off_curve(), g1_off_group(), bytes(inf_bad)]
    pubkeys = [{"pk": c.hex(), "expect": o.pubkey_validate(c)} for c in pk_cases]

    msgs = [hashlib.sha256(b"agg-%d" % i).digest() for i in range(64)]
    sigs = [o.g2_compress(o.sign(sks[i % 8], msgs[i])) for i in range(64)]
    flipped = bytes([sigs[3][0] & 0x7F]) + sigs[3][1:]
    inf_sig = bytes([0xC0]) + bytes(95)
    agg_inputs = [sigs[:1], sigs[:2], sigs[:5], sigs[:64], [],
                  sigs[:3] + [flipped] + sigs[4:6], sigs[:2] + [g2_off_group()], [inf_sig, sigs[7]],
                  sigs[:4] + [bytes(95)]]
    aggs = []
    for inp in agg_inputs:
        code, out = o.signatures_aggregate(inp)
        aggs.append({"sigs": [s.hex() for s in inp], "expect": code, "aggregate": out.hex() if out else None})

    dep = []
    for i in range(4):
        m = hashlib.sha256(b"deposit-%d" % i).digest()
        dep.append((o.g1_compress(pks[i]), m, o.g2_compress(o.sign(sks[i], m))))
    m = hashlib.sha256(b"deposit-x").digest()
    good_sig = o.g2_compress(o.sign(sks[5], m))
    dep += [
        (o.g1_compress(pks[5]), hashlib.sha256(b"other").digest(), good_sig),  # wrong message
        (o.g1_compress(pks[6]), m, good_sig),                                 # wrong key
        (bytes([0xC0]) + bytes(47), m, good_sig),                             # infinity key
        (g1_off_group(), m, good_sig),                                        # key outside G1
        (o.g1_compress(pks[5]), m, bytes([good_sig[0] & 0x7F]) + good_sig[1:]),  # bad signature encoding
        (o.g1_compress(pks[5]), m, g2_off_group()),                           # signature outside G2
    ]
    deposits = [{"pk": a.hex(), "msg": b.hex(), "sig": c.hex(), "expect": int(o.deposit_valid(a, b, c))}
                for a, b, c in dep]
    json.dump({"note": "oracle/bls12381.py pubkey_validate / signatures_aggregate / deposit_valid "
                       "(processDeposit.ts:62-70, chain/opPools signature aggregation); codes are BLST numbers, "
                       "20 = EMPTY_AGGREGATE_ARRAY",
               "pubkeys": pubkeys, "aggregates": aggs, "deposits": deposits}, open(OUT, "w"), indent=0)
    print("pubkeys", [c["expect"] for c in pubkeys])
    print("aggregates", [c["expect"] for c in aggs])
    print("deposits", [c["expect"] for c in deposits])


if __name__ == "__main__":
    main()
