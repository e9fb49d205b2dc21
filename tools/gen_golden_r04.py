"""Round-4 golden fixture: pairing values with injected randomizers (tests/golden/pairing.json).

    python tools/gen_golden_r04.py

SURVEY 8(c) asks for "Miller-loop + final-exp results with injected scalars for deterministic
intermediate checks".  The device's verify kernels compute, per set i of a call,
f_i = MillerLoop(r_i pk_i, H(m_i)) (bgv_debug_prepare returns it), where pk_i is the set's
aggregate pubkey and r_i its batch randomizer (blst's mul_n_aggregate, maybeBatch.ts:18-25).
bgv_debug_prepare injects the randomizers: set i takes the i-th nonzero splitmix64 output w_i
of the call's seed, read as r_i = lo32(w_i) + hi32(w_i) * x^2 mod r (bls_curve.h jac_mul_glv,
DESIGN.md section 1).  The device's f_i is a projectively scaled Miller value (P Jacobian, lines
scaled by Fp2 / Fp factors), so the pinned quantity is the pairing value after the final
exponentiation, which kills those factors:

  sets[i].gt      e(r_i pk_i, H(m_i)) = final_exp(miller_loop(r_i pk_i, H(m_i)))   (576 B)
  sets[i].miller  the oracle's (textbook affine) miller_loop(r_i pk_i, H(m_i))       (576 B)

576-byte values are 12 canonical big-endian Fp coefficients in tower order
[a.c0, a.c1, a.c2, b.c0, b.c1, b.c2] (each Fp2 as re, im), the bgv_debug_prepare format.
The cache layout is tests/golden/keys.json's (index k = interop-style key k).  Signatures are
valid (they do not enter f_i).  Data only: inputs and expected outputs; the oracle is pinned
to the reference's own known answers (tests/test_oracle_kat.py).
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12381 as o  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "pairing.json")
SEED = 0x5EED0004
MASK64 = (1 << 64) - 1


def splitmix64(state):
    state = (state + 0x9E3779B97F4A7C15) & MASK64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return state, z ^ (z >> 31)


def randomizers(seed, n):
    """bgv_api.cpp bgv_debug_prepare: the i-th nonzero splitmix64 word, r = lo + hi x^2 mod r."""
    out, st = [], seed
    while len(out) < n:
        st, w = splitmix64(st)
        if w:
            out.append((w, ((w & 0xFFFFFFFF) + (w >> 32) * o.X_ABS ** 2) % o.R))
    return out


def f12_bytes(f):
    return b"".join(v.to_bytes(48, "big") for v in o.f12_to_tower_list(f))


def main():
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    sks = [int(s, 16) for s in keys["sk"]]
    pks = [o.sk_to_pk(sk) for sk in sks]
    # 8 single sets, then aggregates of 2, 3, 16 (k_pk_agg16 tree) and 40 keys
    shapes = [[k] for k in (0, 1, 2, 7, 31, 64, 100, 127)]
    shapes += [[3, 4], [5, 9, 11], list(range(16, 32)), [(7 * j) % 128 for j in range(40)]]
    rs = randomizers(SEED, len(shapes))
    cases = []
    for i, (idx, (w, r)) in enumerate(zip(shapes, rs)):
        msg = hashlib.sha256(b"pairing-golden-%d" % i).digest()
        agg_sk = sum(sks[k] for k in idx) % o.R
        sig = o.g2_compress(o.sign(agg_sk, msg))
        pk = o.pubkey_aggregate([pks[k] for k in idx])
        h = o.hash_to_g2(msg)
        m = o.miller_loop(o.g1_mul(pk, r), h)
        e = o.final_exp(m)
        assert e == o.pairing(pk, h) if r == 1 else True
        cases.append({"pk_indices": idx, "msg": msg.hex(), "sig": sig.hex(), "word": "%016x" % w,
                      "r": "%064x" % r, "miller": f12_bytes(m).hex(), "gt": f12_bytes(e).hex()})
        print("set", i, "n_pk", len(idx), flush=True)
    json.dump({"note": __doc__.strip().splitlines()[0], "seed": SEED, "sets": cases}, open(OUT, "w"), indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
