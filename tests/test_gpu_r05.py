"""GPU tests added in round 5.

One call over several devices (bgv_set_split; advisor r04): a job big enough to be cut into
per-device runs takes its host-side checks (an index not in the cache, an empty aggregate) on
the whole job before it is cut, so they decide the job ahead of any device status -- an
undecodable signature in an earlier run included -- exactly as in the unsplit call
(bgv_api.cpp job_precheck; the reference raises them before any crypto:
packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39, chain/bls/utils.ts:5-16).  A one-set job
is never cut (bgv_set_split(1) acts as 2).
"""
import hashlib

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
NKEYS = 8192


def _sk(i):
    return (int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R).to_bytes(32, "big")


@pytest.fixture(scope="module")
def ctxs():
    from lodestar_amd import native
    sks = [_sk(i) for i in range(NKEYS)]
    out = []
    for devs in ([0], [0, 0]):
        c = native.Context(devs)
        c.keygen(b"".join(sks), cache_first=0, want_pubkeys=False)
        out.append(c)
    out[1].set_split(2048)
    yield out, sks
    for c in out:
        c.close()


def _sets(c, sks, n):
    from lodestar_amd import native
    roots = [hashlib.sha256(b"r05-split-%d" % i).digest() for i in range(n)]
    sigs = c.sign(b"".join(sks[i] for i in range(n)), b"".join(roots))
    return [native.SetSpec(roots[i], sigs[96 * i:96 * i + 96], pk_indices=[i]) for i in range(n)]


def test_split_host_checks_precede_device_statuses(ctxs):
    from lodestar_amd import native
    (one, two), sks = ctxs
    base = _sets(one, sks, 4096)
    broken = lambda s: native.SetSpec(s.msg, bytes([s.sig[0] & 0x7F]) + s.sig[1:], pk_indices=list(s.pk_indices))
    # undecodable signature early (first device's run), index outside the cache late (second run)
    sets = list(base)
    sets[10] = broken(base[10])
    sets[4000] = native.SetSpec(base[4000].msg, base[4000].sig, pk_indices=[NKEYS + 5])
    got = [c.verify_jobs([(sets, False)], native.MODE_WORKER) for c in (one, two)]
    assert got == [[-native.BGV_E_BAD_INDEX]] * 2
    # an empty aggregate late beats the undecodable signature early too
    sets[4000] = native.SetSpec(base[4000].msg, base[4000].sig, pk_indices=[])
    got = [c.verify_jobs([(sets, False)], native.MODE_WORKER) for c in (one, two)]
    assert got == [[-native.BGV_E_EMPTY_AGGREGATE]] * 2
    # without a host-side condition the first undecodable signature in set order decides
    sets[4000] = broken(base[4000])
    got = [c.verify_jobs([(sets, False)], native.MODE_WORKER) for c in (one, two)]
    assert got == [[-native.BLST_BAD_ENCODING]] * 2
    # and the valid job, and a host-checked job beside small jobs of the same call
    small = [([s], True) for s in base[:300]]
    sets[10] = base[10]
    sets[4000] = native.SetSpec(base[4000].msg, base[4000].sig, pk_indices=[NKEYS + 1])
    for c in (one, two):
        assert c.verify_jobs([(base, False)], native.MODE_WORKER) == [1]
        codes = c.verify_jobs(small + [(sets, False)], native.MODE_WORKER)
        assert codes == [1] * 300 + [-native.BGV_E_BAD_INDEX]


def test_split_min_one_acts_as_two(ctxs):
    from lodestar_amd import native
    (one, two), sks = ctxs
    base = _sets(one, sks, 3000)
    wrong = native.SetSpec(base[1].msg, base[0].sig, pk_indices=[0])
    jobs = [([s], True) for s in base] + [([wrong], True)]
    try:
        two.set_split(1)
        want = one.verify_jobs(jobs, native.MODE_WORKER)
        assert want == [1] * 3000 + [0]
        assert two.verify_jobs(jobs, native.MODE_WORKER) == want
        assert two.verify_jobs([([wrong], False)], native.MODE_WORKER) == [0]
    finally:
        two.set_split(2048)


# ---------------------------------------------------------------------------------------
# Retry of multi-set batchable jobs in a bulk call: jobs inside one group take the pattern
# tests, jobs that straddle two groups the fanout bisection, one job holding two invalid sets,
# three invalid jobs in one group.  Every verdict must equal the job verified alone
# (BGV_MODE_PER_JOB; chain/bls/multithread/worker.ts:76-98).  (Round 5 measured a weighted test
# per failing group in the first pass itself -- equal or slower at the headline, profiles/r05/
# fpw_ab/ -- and dropped it.)
# ---------------------------------------------------------------------------------------
def test_retry_multi_set_jobs_bulk(ctxs):
    from lodestar_amd import native
    (one, _), sks = ctxs
    n = 6000 * 3  # 18,000 sets > BGV_LATENCY_MAX: a bulk batch
    roots = [hashlib.sha256(b"r05-fpw-%d" % (i // 7)).digest() for i in range(n)]
    keys = [i % NKEYS for i in range(n)]
    sigs = one.sign(b"".join(sks[k] for k in keys), b"".join(roots))
    sets = [native.SetSpec(roots[i], sigs[96 * i:96 * i + 96], pk_indices=[keys[i]]) for i in range(n)]
    # wrong messages: one per group at various slots, two in one job, one in a job that straddles
    # groups 20 / 21 (slots 1278..1280 hold sets 1278, 1279 | 1280), three in one group
    for i in (5, 64 * 4 + 63, 64 * 7 + 30, 64 * 9 + 1, 64 * 9 + 2, 1279, 64 * 40 + 3, 64 * 40 + 20,
              64 * 40 + 41, n - 1):
        sets[i] = native.SetSpec(roots[(i + 700) % n], sets[i].sig, pk_indices=list(sets[i].pk_indices))
    jobs = [(sets[3 * j:3 * j + 3], True) for j in range(n // 3)]
    st = native.BgvStats()
    got = one.verify_jobs(jobs, native.MODE_WORKER, stats=st)
    want = one.verify_jobs(jobs, native.MODE_PER_JOB)
    assert got == want
    assert sum(1 for v in got if v != 1) == 9  # ten wrong sets, two of them in one job
    assert st.batch_retries >= 6


# ---------------------------------------------------------------------------------------
# Uniform groups (BGV_GROUP_UNIFORM): in a bulk call the batchable one-set jobs are laid out
# grouped by signing root, and a group whose sets all share one root takes ONE Miller loop over
# its pubkey sum, e(sum_i r_i pk_i, H) = prod_i e(r_i pk_i, H), instead of one per set; a failing
# uniform group gets its slots' own pairs for the retry tests.  Gossip attestations of one
# committee share a root (SURVEY 8(d) "mainnet-shaped").  Every verdict must equal the job
# verified alone (chain/bls/multithread/worker.ts:76-98).
# ---------------------------------------------------------------------------------------
def test_uniform_groups_interleaved_committees(ctxs):
    from lodestar_amd import native
    (one, _), sks = ctxs
    n = 24000
    ncomm = 40  # committees, interleaved in arrival order: the layout regroups them by root
    comm = [(i * 7) % ncomm for i in range(n)]
    roots = [hashlib.sha256(b"r05-uniform-%d" % c).digest() for c in range(ncomm)]
    keys = [(i * 13) % NKEYS for i in range(n)]
    msgs = [roots[c] for c in comm]
    sigs = one.sign(b"".join(sks[k] for k in keys), b"".join(msgs))
    sets = [native.SetSpec(msgs[i], sigs[96 * i:96 * i + 96], pk_indices=[keys[i]]) for i in range(n)]
    want = [1] * n
    # wrong keys keep their committee's root (their uniform group fails and is retried):
    # singles, two in one committee close together, and one beside an undecodable signature;
    # a wrong message is a root of its own
    for i in (3, 4000, 4040, 12345, 23999, 777):
        sets[i] = native.SetSpec(msgs[i], sets[i].sig, pk_indices=[(keys[i] + 1) % NKEYS])
        want[i] = 0
    sets[778] = native.SetSpec(msgs[778], bytes([sets[778].sig[0] & 0x7F]) + sets[778].sig[1:], pk_indices=[keys[778]])
    want[778] = -native.BLST_BAD_ENCODING
    sets[9000] = native.SetSpec(hashlib.sha256(b"other").digest(), sets[9000].sig, pk_indices=[keys[9000]])
    want[9000] = 0
    jobs = [([s], True) for s in sets]
    # a multi-set batchable job and a non-batchable 64-set job ride along
    extra = [(sets[100:103], True), (sets[200:264], False)]
    st = native.BgvStats()
    got = one.verify_jobs(jobs + extra, native.MODE_WORKER, stats=st)
    assert got[:n] == want
    assert got[n:] == [1, 1]
    assert st.batch_retries >= 5
    # the same sets one by one (small calls: the latency path, no uniform groups)
    assert one.verify_jobs(jobs[:64], native.MODE_PER_JOB) == want[:64]


def test_uniform_groups_one_job(ctxs):
    """One non-batchable job of 8192 sets over 16 roots (the epoch sweep's shape): uniform groups
    inside one job; valid, and false with one wrong key."""
    from lodestar_amd import native
    (one, two), sks = ctxs
    n = 8192
    roots = [hashlib.sha256(b"r05-sweep-%d" % (i // 512)).digest() for i in range(n)]
    sigs = one.sign(b"".join(sks[i % NKEYS] for i in range(n)), b"".join(roots))
    sets = [native.SetSpec(roots[i], sigs[96 * i:96 * i + 96], pk_indices=[i % NKEYS]) for i in range(n)]
    for c in (one, two):
        assert c.verify_jobs([(sets, False)], native.MODE_WORKER) == [1]
    bad = list(sets)
    bad[5000] = native.SetSpec(roots[5000], sets[5000].sig, pk_indices=[(5000 + 1) % NKEYS])
    for c in (one, two):
        assert c.verify_jobs([(bad, False)], native.MODE_WORKER) == [0]


def test_uniform_groups_weighted_positions(ctxs):
    """The weighted test of a failing uniform group (BGV_GROUP_WEIGHTED: slot k weighted by k + 1,
    the lone invalid slot named as the w with V^w = W): wrong keys at the first slot of one group
    and the last slot of another (w = 1 and w = 64), one beside an undecodable signature (a dead
    slot, its weight skipped), and two in one group (no w matches: the pattern tests follow).
    Every verdict equals the job verified alone."""
    from lodestar_amd import native
    (one, _), sks = ctxs
    n = 24576
    committee = 256  # four aligned 64-set groups per root
    roots = [hashlib.sha256(b"r05-weighted-%d" % (i // committee)).digest() for i in range(n)]
    keys = [(i * 11) % NKEYS for i in range(n)]
    sigs = one.sign(b"".join(sks[k] for k in keys), b"".join(roots))
    sets = [native.SetSpec(roots[i], sigs[96 * i:96 * i + 96], pk_indices=[keys[i]]) for i in range(n)]
    want = [1] * n
    wrong = [0, 64 * 2 + 63, 64 * 5 + 20, 64 * 9 + 7, 64 * 9 + 50, 64 * 30 + 1]
    for i in wrong:
        sets[i] = native.SetSpec(roots[i], sets[i].sig, pk_indices=[(keys[i] + 1) % NKEYS])
        want[i] = 0
    i = 64 * 5 + 21  # undecodable beside the wrong key of group 5
    sets[i] = native.SetSpec(roots[i], bytes([sets[i].sig[0] & 0x7F]) + sets[i].sig[1:], pk_indices=[keys[i]])
    want[i] = -native.BLST_BAD_ENCODING
    jobs = [([s], True) for s in sets]
    st = native.BgvStats()
    got = one.verify_jobs(jobs, native.MODE_WORKER, stats=st)
    assert got == want
    assert st.batch_retries >= 5
