"""GPU: the batch-fail -> per-job retry (worker.ts:76-98) with pattern tests.

A failing first-pass group whose jobs all lie inside it is retried in one round by tests
S_j = {jobs whose index has bit j set}; the complement's verdict comes from the group's
pairing value (bgv_api.cpp PatternUnit).  Every job's code must still be its own
verdict: 1 valid, 0 invalid, for every placement of invalid jobs -- one, two that differ
in one or several bits, the first and last job, every job, groups of non-power-of-two
size, several groups -- and for jobs that span groups (not pattern-testable: fanout
bisection).  Checked against the per-job mode (each job verified alone).
"""
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


@pytest.fixture(scope="module")
def env():
    from lodestar_amd import native
    keys = json.load(open(os.path.join(GOLD, "keys.json")))
    c = native.Context()
    c.pubkeys_put(0, b"".join(bytes.fromhex(k) for k in keys["pk_compressed"]), native.PK_COMPRESSED)
    sks = [int(s, 16) for s in keys["sk"]]
    yield c, sks
    c.close()


def _sets(ctx, sks, n, tag):
    from lodestar_amd import native
    msgs = [hashlib.sha256(tag + i.to_bytes(4, "little")).digest() for i in range(n)]
    key = [(3 * i + 1) % len(sks) for i in range(n)]
    sigs = ctx.sign(b"".join(sks[k].to_bytes(32, "big") for k in key), b"".join(msgs))
    return [native.SetSpec(msgs[i], sigs[96 * i:96 * i + 96], pk_indices=[key[i]]) for i in range(n)]


def _corrupt(s):
    from lodestar_amd import native
    return native.SetSpec(hashlib.sha256(b"wrong" + s.msg).digest(), s.sig, pk_indices=s.pk_indices)


@pytest.mark.parametrize("n,bad", [
    (64, [5]), (64, [5, 6]), (64, [0, 63]), (64, [1, 2, 4, 8]), (64, [9, 54]), (64, list(range(64))),
    (64, []), (37, [36]), (37, [0, 17, 33]), (2, [1]), (130, [3, 70, 129]), (200, [64, 65, 127, 128, 199]),
])
def test_pattern_retry_one_set_jobs(env, n, bad):
    from lodestar_amd import native
    ctx, sks = env
    sets = _sets(ctx, sks, n, b"retry-%d-" % n)
    for i in bad:
        sets[i] = _corrupt(sets[i])
    jobs = [([s], True) for s in sets]
    want = [0 if i in bad else 1 for i in range(n)]
    st = native.BgvStats()
    assert ctx.verify_jobs(jobs, native.MODE_WORKER, st) == want
    assert st.batch_retries == len({i // 64 for i in bad})
    assert ctx.verify_jobs(jobs, native.MODE_PER_JOB) == want


def test_retry_jobs_spanning_groups(env):
    """Jobs of 1-3 sets: some straddle a 64-slot group (fanout bisection), the rest are
    pattern-tested; invalid sets in straddling and contained jobs."""
    from lodestar_amd import native
    ctx, sks = env
    sizes = [1 + (i % 3) for i in range(70)]
    sets = _sets(ctx, sks, sum(sizes), b"retry-span-")
    jobs, pos = [], 0
    for n in sizes:
        jobs.append([sets[pos + k] for k in range(n)])
        pos += n
    bad_jobs = {4, 21, 22, 40, 69}
    for j in bad_jobs:
        jobs[j][-1] = _corrupt(jobs[j][-1])
    calls = [(js, True) for js in jobs]
    want = [0 if j in bad_jobs else 1 for j in range(len(jobs))]
    assert ctx.verify_jobs(calls, native.MODE_WORKER) == want
    assert ctx.verify_jobs(calls, native.MODE_PER_JOB) == want


def test_pattern_retry_with_undecodable_and_mixed(env):
    """A group with an undecodable signature (rejects on its own, not live in the product),
    a wrong-key set and a wrong-message set among valid one-set jobs."""
    from lodestar_amd import native
    ctx, sks = env
    sets = _sets(ctx, sks, 64, b"retry-mixed-")
    sets[7] = native.SetSpec(sets[7].msg, bytes([sets[7].sig[0] & 0x7F]) + sets[7].sig[1:], pk_indices=sets[7].pk_indices)
    sets[20] = native.SetSpec(sets[20].msg, sets[20].sig, pk_indices=[(sets[20].pk_indices[0] + 1) % len(sks)])
    sets[41] = _corrupt(sets[41])
    want = [1] * 64
    want[7], want[20], want[41] = -native.BLST_BAD_ENCODING, 0, 0
    jobs = [([s], True) for s in sets]
    assert ctx.verify_jobs(jobs, native.MODE_WORKER) == want
    assert ctx.verify_jobs(jobs, native.MODE_PER_JOB) == want
