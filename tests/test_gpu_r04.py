"""GPU tests added in round 4.

Pubkey cache writes (VERDICT r03 "next" #6, advisor r03): bgv_pubkeys_put decodes into staging
memory and publishes an append without waiting for running verifies; an undecodable record
commits its run with the index marked (sets naming it reject BGV_E_BAD_INDEX), a gap writes
nothing, a later put over the index clears the mark.  Reference: EpochContext.addPubkey
(packages/state-transition/src/cache/epochContext.ts:702-705), pubkeyCache.ts:56-77.
"""
import json
import os
import threading
import time

import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return json.load(open(os.path.join(GOLD, name)))


def test_pubkeys_put_marks_undecodable_and_appends():
    from lodestar_amd import native
    keys = [bytes.fromhex(k) for k in load("keys.json")["pk_compressed"]]
    sig_cases = load("signatures.json")["cases"]
    c = native.Context()
    try:
        c.pubkeys_put(0, b"".join(keys[:4]))
        # a run with an undecodable record in the middle: committed, index 5 marked
        with pytest.raises(native.BlsGpuError) as e:
            c.pubkeys_put(4, keys[4] + bytes(48) + keys[6])
        assert "BLST_BAD_ENCODING" in str(e.value)
        assert c.pubkeys_count() == 7
        # a gap writes nothing
        with pytest.raises(native.BlsGpuError):
            c.pubkeys_put(9, keys[9])
        assert c.pubkeys_count() == 7

        def job(k):
            s = next(x for x in sig_cases if x["key"] == k)
            return ([native.SetSpec(bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]), pk_indices=[k])], True)

        codes = c.verify_jobs([job(4), job(6)], native.MODE_WORKER)
        assert codes == [1, 1]
        s5 = next(x for x in sig_cases if x["key"] == 5)
        bad = ([native.SetSpec(bytes.fromhex(s5["msg"]), bytes.fromhex(s5["sig"]), pk_indices=[5])], True)
        assert c.verify_jobs([bad], native.MODE_WORKER) == [-native.BGV_E_BAD_INDEX]
        # overwriting the marked index with the real key clears the mark
        c.pubkeys_put(5, keys[5])
        assert c.verify_jobs([bad], native.MODE_WORKER) == [1]
    finally:
        c.close()


def test_pubkeys_append_while_verifying():
    """Appends of 65,536 keys interleaved with verify calls on another thread: every call
    completes with the right verdict and the appended keys verify afterwards."""
    from lodestar_amd import native
    keys = [bytes.fromhex(k) for k in load("keys.json")["pk_compressed"]]
    sig_cases = load("signatures.json")["cases"]
    c = native.Context()
    try:
        keys = keys[:128]
        c.pubkeys_put(0, b"".join(keys))
        s = next(x for x in sig_cases if x["key"] == 3)
        job = ([native.SetSpec(bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]), pk_indices=[3])], True)
        stop = threading.Event()
        results, lat = [], []

        def verifier():
            while not stop.is_set():
                t = time.perf_counter()
                results.append(c.verify_jobs([job] * 64, native.MODE_WORKER))
                lat.append(time.perf_counter() - t)

        th = threading.Thread(target=verifier)
        th.start()
        n0 = len(keys)
        block = b"".join(keys) * 64  # 8192 keys per put (the 128 keys repeated)
        for k in range(8):
            c.pubkeys_put(n0 + 8192 * k, block)
        stop.set()
        th.join()
        assert results and all(r == [1] * 64 for r in results)
        assert c.pubkeys_count() == n0 + 65536
        idx = n0 + 65536 - 128 + 3  # the last block's copy of key 3
        j = ([native.SetSpec(bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]), pk_indices=[idx])], True)
        assert c.verify_jobs([j], native.MODE_WORKER) == [1]
    finally:
        c.close()
