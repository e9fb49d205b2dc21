"""The C++ CPU restatement (oracle/cpu/blscpu.cpp, the cpu_baseline of bench.py)
pinned to the Python oracle's golden vectors: hash_to_G2 bytes and every verdict
vector, in worker (batch + retry) and per-job modes."""
import json
import os

import pytest

from oracle import bls12381 as o

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def C():
    from oracle.cpu import blscpu
    blscpu.lib()
    return blscpu


def test_hash_to_g2_golden(C):
    for c in json.load(open(os.path.join(GOLD, "hash_to_g2.json")))["cases"]:
        assert C.hash_to_g2(bytes.fromhex(c["msg"])).hex() == c["uncompressed"]


def test_sk_to_pk(C):
    keys = json.load(open(os.path.join(GOLD, "keys.json")))
    pks = C.sk_to_pk96(b"".join(bytes.fromhex(s) for s in keys["sk"][:16]))
    for i in range(16):
        assert pks[96 * i:96 * i + 96].hex() == keys["pk_uncompressed"][i]


@pytest.mark.parametrize("mode", [0, 1])
def test_verdict_vectors(C, mode):
    keys = json.load(open(os.path.join(GOLD, "keys.json")))
    pk = [o.g1_deserialize(bytes.fromhex(k)) for k in keys["pk_uncompressed"]]
    jobs, exp = [], []
    for jb in json.load(open(os.path.join(GOLD, "verdicts.json")))["jobs"]:
        sets = []
        for s in jb["sets"]:
            agg = o.g1_serialize(o.pubkey_aggregate([pk[i] for i in s["pk"]])) if s["pk"] else None
            sets.append((agg, bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"])))
        jobs.append((sets, jb["batchable"]))
        exp.append(jb["expect"])
    assert C.verify_jobs(jobs, mode, threads=2) == exp


@pytest.mark.parametrize("n", [7, 8, 9, 16])
def test_multi_pair_groups(C, n):
    """Jobs whose Miller loops span whole and partial 8-pair groups (the sig-sum pair
    lands in the last group or a group of its own); one wrong set turns the job false
    and the retry isolates nothing else (worker mode splits the 1-set jobs)."""
    keys = json.load(open(os.path.join(GOLD, "keys.json")))
    cases = json.load(open(os.path.join(GOLD, "signatures.json")))["cases"]
    pk = [bytes.fromhex(k) for k in keys["pk_uncompressed"]]
    sets = [(pk[c["key"]], bytes.fromhex(c["msg"]), bytes.fromhex(c["sig"])) for c in cases[:n]]
    bad = list(sets)
    bad[n // 2] = (sets[n // 2][0], sets[(n // 2) + 1 - n][1], sets[n // 2][2])
    jobs = [(sets, True), (bad, True)] + [([s], True) for s in bad]
    exp = [1, 0] + [0 if i == n // 2 else 1 for i in range(n)]
    assert C.verify_jobs(jobs, 0, threads=2) == exp
    assert C.verify_jobs(jobs, 1, threads=2) == exp
