"""Driver of tools/ubench_rns.hip: writes a random Fp12 value, runs the latency benchmark and
checks the values it returns against the oracle (the RNS engine's chain, its fp_t input
conversion, and the current eight-part engine's chain).  Prints the benchmark's JSON lines and
one verdict line.

    python tools/gpu/rns_probe.py [calls] [seed]
"""
import json
import os
import random
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_rns as g  # noqa: E402
from oracle import bls12381 as o  # noqa: E402

R28 = 1 << 392


def limbs28(v):
    return [(v >> (28 * k)) & ((1 << 28) - 1) for k in range(14)]


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    rnd = random.Random(seed)
    a = tuple((rnd.randrange(g.P), rnd.randrange(g.P)) for _ in range(6))
    words = []
    for k in range(6):
        for e in range(2):
            words += g.to_rns(a[k][e] * g.M % g.P)
    for k in range(6):
        for e in range(2):
            words += limbs28(a[k][e] * R28 % g.P)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        open(fin, "wb").write(struct.pack("<%dI" % len(words), *words))
        exe = os.path.join(ROOT, "tools", "bin", "ubench_rns")
        res = subprocess.run([exe, fin, fout, str(calls)], capture_output=True, text=True, timeout=120)
        sys.stdout.write(res.stdout)
        if res.returncode != 0:
            sys.stderr.write(res.stderr)
            sys.exit(res.returncode)
        raw = open(fout, "rb").read()
    out = struct.unpack("<%dI" % (len(raw) // 4), raw)
    rns_chain = [list(out[30 * c:30 * c + 30]) for c in range(12)]
    from_fp = [list(out[360 + 30 * c:360 + 30 * c + 30]) for c in range(12)]
    p8 = out[720:720 + 168]
    tofp = out[720 + 168:]
    want = a
    for _ in range(calls):
        want = o.f12_conj(o.f12_pow(want, o.X_ABS))
    got_rns = g.rns_to_f12(rns_chain)
    got_from = g.rns_to_f12(from_fp)
    rinv = pow(R28, -1, g.P)
    vals = []
    for c in range(12):
        v = sum(p8[14 * c + q] << (28 * q) for q in range(14))
        vals.append(v * rinv % g.P)
    got_p8 = tuple((vals[2 * k], vals[2 * k + 1]) for k in range(6))
    tv = []
    for c in range(12):
        v = sum(tofp[14 * c + q] << (28 * q) for q in range(14))
        assert v < 2 * g.P, "to_fp output not below 2p"
        tv.append(v * rinv % g.P)
    got_tofp = tuple((tv[2 * k], tv[2 * k + 1]) for k in range(6))
    bounds = max(g.rns_int(r) for r in rns_chain) / g.P
    verdict = {"rns_chain_ok": got_rns == want, "rns_from_fp_ok": got_from == a, "part8_chain_ok": got_p8 == want,
               "rns_to_fp_ok": got_tofp == a,
               "rns_output_bound_p": round(bounds, 3), "calls": calls, "seed": seed}
    print(json.dumps(verdict))
    sys.exit(0 if verdict["rns_chain_ok"] and verdict["rns_from_fp_ok"] and verdict["part8_chain_ok"] and verdict["rns_to_fp_ok"] else 1)


if __name__ == "__main__":
    main()
