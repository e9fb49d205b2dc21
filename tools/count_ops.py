"""Count Fp products per verify-kernel per set (roofline numerator).

Builds tests/native/hostsim.cpp with -DBGV_COUNT_OPS (the kernels' own per-lane
math compiled for the host with a counter in fp_mul / fp_sqr), runs each
kernel body once on representative inputs and writes profiles/opcounts.json.
Random-scalar steps are averaged over seeded 64-bit scalars.

    python tools/count_ops.py
"""
import ctypes
import hashlib
import json
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12381 as o  # noqa: E402
from tests import hostsim as hs  # noqa: E402

LIB = os.path.join(ROOT, "tests", "native", "libhostsim_count.so")


def main():
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-DBGV_COUNT_OPS", "-o", LIB,
                           os.path.join(ROOT, "tests", "native", "hostsim.cpp")])
    L = ctypes.CDLL(LIB)
    L.hs_count_mul.restype = ctypes.c_ulonglong
    L.hs_count_sqr.restype = ctypes.c_ulonglong

    def count(fn):
        L.hs_count_reset()
        fn()
        return int(L.hs_count_mul()), int(L.hs_count_sqr())

    rng = random.Random(7)
    sk = o.interop_secret_key(3)
    pk = o.sk_to_pk(sk)
    msg = hashlib.sha256(b"count").digest()
    sig = o.sign(sk, msg)
    out = {}
    trials = 8
    acc = [0, 0]
    for _ in range(trials):
        m, s = count(lambda: L.hs_k_sig_body(o.g2_compress(sig), ctypes.c_uint64(rng.getrandbits(64) | 1)))
        acc[0] += m
        acc[1] += s
    out["k_sig"] = [acc[0] / trials, acc[1] / trials]
    out["k_hash"] = list(count(lambda: L.hs_k_hash_body(msg)))
    for npk in (1, 128):
        acc = [0, 0]
        for _ in range(trials):
            m, s = count(lambda: L.hs_k_pk_body(hs.g1_b(pk), npk, ctypes.c_uint64(rng.getrandbits(64) | 1)))
            acc[0] += m
            acc[1] += s
        out["k_pk[n_pk=%d]" % npk] = [acc[0] / trials, acc[1] / trials]
    h = o.hash_to_g2(msg)
    out["k_miller"] = list(count(lambda: L.hs_k_miller_body(hs.g1_b(pk), hs.g2_b(h))))
    sig2 = o.sign(o.interop_secret_key(4), msg)
    out["k_final[group sig pair]"] = list(count(lambda: L.hs_k_group_miller_body(hs.g2_b(sig))))
    out["k_final[per slot sig add]"] = list(count(lambda: L.hs_k_group_add_body(hs.g2_b(sig), hs.g2_b(sig2))))
    f12 = hs.fp12_b_tower([rng.randrange(o.P) for _ in range(12)])
    out["k_final[per group]"] = list(count(lambda: L.hs_k_final_body(f12)))
    out["k_final[per product step]"] = list(count(lambda: L.hs_k_product_step(f12)))
    res = {
        "note": "Fp products [mul, sqr] per set (per group / per group-product step where named), counted in the "
                "kernels' own math (host build, -DBGV_COUNT_OPS). Team (k_final) work is counted as the one-lane "
                "tower operations it replaces. Fp-mul-eq = mul + sqr; "
                "algorithmic u32 MACs per Fp-mul-eq = 288 (12x32-bit CIOS: 144 product + 144 reduction).",
        "macs_per_fp_mul": 288,
        "counts": out,
        "fp_mul_eq": {k: v[0] + v[1] for k, v in out.items()},
    }
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "profiles", "opcounts.json"), "w"), indent=1)
    print(json.dumps(res["fp_mul_eq"], indent=1))


if __name__ == "__main__":
    main()
