"""GPU tests added in round 6.

Retry rounds of uniform groups just above the latency bound (advisor r05, high): a bulk call
whose first pass is uniform (nslots + ngroups > BGV_LATENCY_MAX, one Miller loop per group over
its pubkey sum) runs retry rounds with only a few test groups, so nslots + nrg can fall below
the bound.  The closing must still be k_final12 (it multiplies the tests' pubkey-sum pairs);
k_final_fold would multiply the uniform groups' unwritten per-slot f_i and reject valid jobs.
Every verdict must equal the job verified alone (chain/bls/multithread/worker.ts:76-98).
"""
import hashlib

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
NKEYS = 4096


def _sk(i):
    return (int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R).to_bytes(32, "big")


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd import native
    sks = [_sk(i) for i in range(NKEYS)]
    c = native.Context([0])
    c.keygen(b"".join(sks), cache_first=0, want_pubkeys=False)
    yield c, sks
    c.close()


@pytest.mark.parametrize("n", [16100, 16200, 16300])
def test_uniform_retry_just_above_latency_bound(ctx, n):
    from lodestar_amd import native
    c, sks = ctx
    committee = 128
    roots = [hashlib.sha256(b"r06-window-%d" % (i // committee)).digest() for i in range(n)]
    keys = [(i * 7) % NKEYS for i in range(n)]
    sigs = c.sign(b"".join(sks[k] for k in keys), b"".join(roots))
    sets = [native.SetSpec(roots[i], sigs[96 * i:96 * i + 96], pk_indices=[keys[i]]) for i in range(n)]
    want = [1] * n
    for i in (1, 64 * 3 + 17, 64 * 40 + 63, n - 2):  # one wrong key per failing group
        sets[i] = native.SetSpec(roots[i], sets[i].sig, pk_indices=[(keys[i] + 1) % NKEYS])
        want[i] = 0
    jobs = [([s], True) for s in sets]
    st = native.BgvStats()
    got = c.verify_jobs(jobs, native.MODE_WORKER, stats=st)
    assert got == want
    assert st.batch_retries >= 4
