"""BASELINE.json configurations at full size on the GPU, checked through
properties that do not need the oracle at that size: every verdict is known by
construction (device-signed with interop keys, then corrupted in known places),
aggregate signatures are signatures by the summed secret key, and the pubkey
aggregates are pinned against the oracle on a few committees.

  config 1  128 single sets, one job, per-job mode (BlsSingleThreadVerifier)
  config 2  1024 aggregate sets x 128 distinct pubkeys (contiguous committees), 8 x 128-set jobs
  config 4  8192 batchable one-set jobs, 1 % corrupted (random.Random(0x8192).sample), and one call
  config 5  one rank's shard of the epoch sweep: a 1,048,576-key device cache, 131,072 single sets
"""
import hashlib
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def interop_sk_int(i):
    """state-transition/src/util/interop.ts:19-22"""
    return int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R


def sk_bytes(k):
    return k.to_bytes(32, "big")


@pytest.fixture(scope="module")
def big():
    """Context with 1,048,576 interop validators in the device cache."""
    from lodestar_amd import native
    c = native.Context()
    n = 1 << 20
    sks = [interop_sk_int(i) for i in range(n)]
    for lo in range(0, n, 1 << 17):
        c.keygen(b"".join(sk_bytes(k) for k in sks[lo:lo + (1 << 17)]), cache_first=lo, want_pubkeys=False)
    assert c.pubkeys_count() == n
    yield c, sks
    c.close()


def test_config1_single_thread_job(big):
    from lodestar_amd import native
    c, sks = big
    idx = list(range(1000, 1128))
    msgs = [hashlib.sha256(b"config1-%d" % i).digest() for i in idx]
    sigs = c.sign(b"".join(sk_bytes(sks[i]) for i in idx), b"".join(msgs))
    sets = [native.SetSpec(msgs[j], sigs[96 * j:96 * j + 96], pk_indices=[i]) for j, i in enumerate(idx)]
    assert c.verify_jobs([(sets, False)], native.MODE_PER_JOB) == [1]
    sets[77] = native.SetSpec(msgs[76], sets[77].sig, pk_indices=[idx[77]])
    assert c.verify_jobs([(sets, False)], native.MODE_PER_JOB) == [0]


def test_config2_aggregates(big):
    """1024 committees of 128 contiguous validators; committee c signs root_c with
    sum(sk) mod r.  Jobs of 128 sets (multithread/index.ts:155-166)."""
    from lodestar_amd import native
    from oracle import bls12381 as o  # pins two pubkey aggregates
    c, sks = big
    ncomm, size = 1024, 128
    roots = [hashlib.sha256(b"lodestar-bench" + c_.to_bytes(4, "little")).digest() for c_ in range(ncomm)]
    agg_sk = [sum(sks[size * q:size * q + size]) % R for q in range(ncomm)]
    sigs = c.sign(b"".join(sk_bytes(k) for k in agg_sk), b"".join(roots))
    for q in (0, 777):
        members = list(range(size * q, size * q + size))
        assert c.aggregate_pubkeys(members) == o.g1_serialize(o.sk_to_pk(agg_sk[q]))
    sets = [native.SetSpec(roots[q], sigs[96 * q:96 * q + 96], pk_indices=list(range(size * q, size * q + size)))
            for q in range(ncomm)]
    jobs = [(sets[j:j + 128], True) for j in range(0, ncomm, 128)]
    assert c.verify_jobs(jobs, native.MODE_WORKER) == [1] * 8
    # a committee missing one member -> its job false; the other 7 true (retry isolates it)
    q = 300
    sets[q] = native.SetSpec(roots[q], sets[q].sig, pk_indices=list(range(size * q, size * q + size - 1)))
    jobs = [(sets[j:j + 128], True) for j in range(0, ncomm, 128)]
    assert c.verify_jobs(jobs, native.MODE_WORKER) == [1, 1, 0, 1, 1, 1, 1, 1]


def _gossip(c, sks, n, base, seed, committee=1):
    """n one-set jobs, 1 % corrupted; `committee` consecutive sets share one signing root
    (mainnet-shaped: one root per committee) -- 1 = distinct roots."""
    from lodestar_amd import native
    key_of = [(base + i * 7919) % len(sks) for i in range(n)]
    msgs = [hashlib.sha256(b"lodestar-bench" + (i // committee).to_bytes(4, "little")).digest() for i in range(n)]
    sigs = c.sign(b"".join(sk_bytes(sks[k]) for k in key_of), b"".join(msgs))
    sigs = [sigs[96 * i:96 * i + 96] for i in range(n)]
    expect = [1] * n
    bad = random.Random(seed).sample(range(n), int(round(n * 0.01)))
    # the undecodable third cycles through a flipped compression flag and the verdict goldens'
    # off-curve and not-in-G2 encodings (invalid or off-curve encodings)
    gold = {j["name"]: j for j in json.load(open(os.path.join(GOLD, "verdicts.json")))["jobs"]}
    undecodable = [(bytes.fromhex(gold["off_curve"]["sets"][0]["sig"]), -2),
                   (bytes.fromhex(gold["not_in_g2"]["sets"][0]["sig"]), -3)]
    for j, i in enumerate(bad):
        if j % 3 == 0:
            msgs[i] = hashlib.sha256(b"wrong" + msgs[i]).digest()
            expect[i] = 0
        elif j % 3 == 1:
            key_of[i] = (key_of[i] + 1) % len(sks)
            expect[i] = 0
        elif (j // 3) % 3 == 0:
            sigs[i] = bytes([sigs[i][0] & 0x7F]) + sigs[i][1:]
            expect[i] = -1
        else:
            sigs[i], expect[i] = undecodable[(j // 3) % 3 - 1]
    sets = [native.SetSpec(msgs[i], sigs[i], pk_indices=[key_of[i]]) for i in range(n)]
    return sets, expect


def test_config4_gossip_8192(big):
    from lodestar_amd import native
    c, sks = big
    sets, expect = _gossip(c, sks, 8192, 0, 0x8192)
    st = native.BgvStats()
    assert c.verify_jobs([([s], True) for s in sets], native.MODE_WORKER, st) == expect
    assert st.batch_retries > 0
    assert {-1, -2, -3} <= set(expect)
    # mode (ii): one call holding all 8192 sets -> rejects with the first error code in set order
    first = next(e for e in expect if e < 0)
    assert c.verify_jobs([(sets, True)], native.MODE_WORKER) == [first]


def _block_import_sets(c, sks, att_size=128):
    """config 3 as chain/blocks/verifyBlocksSignatures.ts:34 sends it: randao (single),
    128 aggregate attestations of att_size distinct validators, one 512-key sync-committee
    aggregate and the proposer (single); aggregate signatures sign with the summed key."""
    import hashlib as _h
    from lodestar_amd import native
    groups = [[7]] + [list(range(att_size * a, att_size * a + att_size)) for a in range(128)]
    groups += [list(range(600000, 600000 + 512)), [11]]
    msgs = [_h.sha256(b"block-import-%d" % i).digest() for i in range(len(groups))]
    agg = [sum(sks[k] for k in g) % R for g in groups]
    sigs = c.sign(b"".join(sk_bytes(k) for k in agg), b"".join(msgs))
    return [native.SetSpec(msgs[i], sigs[96 * i:96 * i + 96], pk_indices=g) for i, g in enumerate(groups)], groups


@pytest.mark.parametrize("n,committee", [(20000, 125), (20000, 1), (96, 16)])
def test_mainnet_shaped_roots(big, n, committee):
    """Sets sharing signing roots: the bulk k_prep hashes each distinct root of a call once
    (bgv_dslot.hsrc / b.uniq) and every slot's Miller loop reads its root's H; the latency
    path (96 sets) hashes every slot.  A corrupted message is a root of its own.  Verdicts by
    construction, both modes."""
    from lodestar_amd import native
    c, sks = big
    sets, expect = _gossip(c, sks, n, 777, 0x5EED + committee, committee)
    assert c.verify_jobs([([s], True) for s in sets], native.MODE_WORKER) == expect
    if n <= 1024:
        assert c.verify_jobs([([s], True) for s in sets], native.MODE_PER_JOB) == expect
    # one non-batchable job of the first 128 sets: valid iff none of them is corrupted
    head = sets[:128]
    neg = [e for e in expect[:128] if e < 0]  # the first undecodable signature in set order decides
    want = neg[0] if neg else (0 if 0 in expect[:128] else 1)
    assert c.verify_jobs([(head, False)], native.MODE_WORKER) == [want]


def test_config3_block_import_full_shape(big):
    """One non-batchable call of 131 sets (16,898 pubkeys aggregated on the device); a
    corrupted attestation signature, a sync aggregate missing a member and a bad encoding
    each turn the call false / reject, as the reference's single job does (no retry)."""
    from lodestar_amd import native
    c, sks = big
    sets, groups = _block_import_sets(c, sks)
    assert len(sets) == 131 and sum(len(g) for g in groups) == 16898
    assert c.verify_jobs([(sets, False)], native.MODE_WORKER) == [1]
    assert c.verify_jobs([(sets, False)], native.MODE_PER_JOB) == [1]
    bad = list(sets)
    bad[40] = native.SetSpec(sets[40].msg, sets[41].sig, pk_indices=groups[40])  # another attestation's sig
    assert c.verify_jobs([(bad, False)], native.MODE_WORKER) == [0]
    bad = list(sets)
    bad[129] = native.SetSpec(sets[129].msg, sets[129].sig, pk_indices=groups[129][:-1])  # sync member missing
    assert c.verify_jobs([(bad, False)], native.MODE_WORKER) == [0]
    bad = list(sets)
    bad[3] = native.SetSpec(sets[3].msg, bytes([sets[3].sig[0] & 0x7F]) + sets[3].sig[1:], pk_indices=groups[3])
    assert c.verify_jobs([(bad, False)], native.MODE_WORKER) == [-native.BLST_BAD_ENCODING]
    # the 512-key attestation variant of SURVEY 8(d) config 3
    sets512, _ = _block_import_sets(c, sks, att_size=512)
    assert c.verify_jobs([(sets512, False)], native.MODE_WORKER) == [1]


def test_config5_aggregate_variant_2048x512(big):
    """Config 5's aggregate variant: 2048 aggregates of 512 validators (the whole 2^20-key
    cache), chunked into 128-set batchable jobs as the pool does (index.ts:155-166); one
    aggregate signed over a wrong root fails its job alone."""
    from lodestar_amd import native
    c, sks = big
    n, size = 2048, 512
    roots = [hashlib.sha256(b"config5-agg-%d" % q).digest() for q in range(n)]
    agg = [sum(sks[size * q:size * q + size]) % R for q in range(n)]
    sigs = c.sign(b"".join(sk_bytes(k) for k in agg), b"".join(roots))
    sets = [native.SetSpec(roots[q], sigs[96 * q:96 * q + 96], pk_indices=range(size * q, size * q + size))
            for q in range(n)]
    jobs = [(sets[j:j + 128], True) for j in range(0, n, 128)]
    assert c.verify_jobs(jobs, native.MODE_WORKER) == [1] * 16
    q = 1500
    sets[q] = native.SetSpec(roots[q - 1], sets[q].sig, pk_indices=range(size * q, size * q + size))
    jobs = [(sets[j:j + 128], True) for j in range(0, n, 128)]
    want = [1] * 16
    want[q // 128] = 0
    assert c.verify_jobs(jobs, native.MODE_WORKER) == want


def test_config5_shard_of_epoch_sweep(big):
    """Rank 0's 131,072 of 1,048,576 sets over the full 2^20-key cache (indices spread
    over all of it), 1 % corrupted; verdicts by construction.  One super-batch of 131,072
    slots: its 2,048 group pairs run on k_miller_team beside two full k_miller rounds
    (bgv_launch_miller's round split)."""
    from lodestar_amd import native
    c, sks = big
    sets, expect = _gossip(c, sks, 1 << 17, 12345, 0x5)
    assert c.verify_jobs([([s], True) for s in sets], native.MODE_WORKER) == expect
