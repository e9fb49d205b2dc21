"""Multi-process verification on the device, two ranks sharing GPU 0
under gloo (the driver's multi-GPU runs use one rank per GPU with RCCL; the protocol is the
same).  Config 4 at full size (8192 sets):

* mode (ii), one call holding all 8192 sets: the job's sets are split over the ranks, each
  rank's Fp12 Miller-loop partial (bgv_verify_partial, 576 B) is all-gathered and one final
  exponentiation (bgv_final_verify) decides; the code equals the single-rank bgv_verify of
  the same job for a valid batch, a wrong message (false) and a bad encoding (rejects);
* mode (i), 8192 batchable one-set jobs with 1 % corrupted: the fast path (one final
  exponentiation over all partials, failing shards re-verified per job) gives the same
  per-job codes as one rank.

Also bgv_init over a device list: [0, 0] (two device records on one GPU) verifies like
[0]; an index past the device count is rejected.
"""
import hashlib
import os
import random
import socket

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N = 8192


def _sk(i):
    return (int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R).to_bytes(32, "big")


def _batch(ctx, native, kind):
    msgs = [hashlib.sha256(b"dist-%d" % i).digest() for i in range(N)]
    sigs = ctx.sign(b"".join(_sk(i) for i in range(N)), b"".join(msgs))
    sigs = [sigs[96 * i:96 * i + 96] for i in range(N)]
    expect = [1] * N
    if kind == "wrong_msg":
        msgs[5000] = hashlib.sha256(b"other").digest()
    elif kind == "bad_encoding":
        sigs[6000] = bytes([sigs[6000][0] & 0x7F]) + sigs[6000][1:]
    elif kind == "corrupt_1pct":
        for j, i in enumerate(random.Random(0x8192).sample(range(N), 82)):
            if j % 3 == 0:
                msgs[i] = hashlib.sha256(b"wrong" + msgs[i]).digest()
                expect[i] = 0
            elif j % 3 == 1:
                sigs[i] = sigs[(i + 1) % N]
                expect[i] = 0
            else:
                sigs[i] = bytes([sigs[i][0] & 0x7F]) + sigs[i][1:]
                expect[i] = -1
    return [native.SetSpec(msgs[i], sigs[i], pk_indices=[i]) for i in range(N)], expect


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lodestar_amd import native
        from lodestar_amd.shard import ShardedVerify
        ctx = native.Context([0])
        ctx.keygen(b"".join(_sk(i) for i in range(N)), cache_first=0, want_pubkeys=False)
        sv = ShardedVerify(ctx.verify_jobs, dist, partial_fn=ctx.verify_partial, final_fn=ctx.final_verify,
                           fast_path=True)
        res = {}
        for kind in ("valid", "wrong_msg", "bad_encoding"):
            sets, _ = _batch(ctx, native, kind)
            single = ctx.verify_jobs([(sets, True)], native.MODE_WORKER)[0]
            res[kind] = (sv.verify_one_job(sets), single)
        sets, expect = _batch(ctx, native, "corrupt_1pct")
        jobs = [([s], True) for s in sets]
        res["mode_i_fast_path"] = (sv(jobs) == expect, True)
        sets, expect = _batch(ctx, native, "valid")
        res["mode_i_all_valid"] = (sv([([s], True) for s in sets]) == expect, True)
        ctx.close()
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001
        q.put((rank, {"error": (repr(e), None)}))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_share_one_job_and_many_jobs():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(60)
    for rank, r in res.items():
        assert "error" not in r, (rank, r)
        assert r["valid"] == (1, 1), r
        assert r["wrong_msg"] == (0, 0), r
        assert r["bad_encoding"] == (-1, -1), r
        assert r["mode_i_fast_path"][0] and r["mode_i_all_valid"][0], r


def test_multi_device_init_on_one_gpu():
    from lodestar_amd import native
    n = native.load().bgv_device_count()
    msgs = [bytes([i + 1]) * 32 for i in range(3)]
    sks = b"".join(bytes([i + 1]) * 32 for i in range(3))
    for devs in ([0], [0, 0], list(range(n))):
        c = native.Context(devs)
        c.keygen(sks, cache_first=0, want_pubkeys=False)  # replicated on every device record
        sigs = c.sign(sks, b"".join(msgs))
        sets = [native.SetSpec(msgs[i], sigs[96 * i:96 * i + 96], pk_indices=[i]) for i in range(3)]
        bad = native.SetSpec(msgs[0], sigs[96:192], pk_indices=[0])
        # several concurrent calls spread over the device records' dispatchers
        import threading
        out = {}

        def call(k):
            out[k] = c.verify_jobs([(sets, True), ([bad], True)])

        th = [threading.Thread(target=call, args=(k,)) for k in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert all(v == [1, 0] for v in out.values()) and len(out) == 6, (devs, out)
        c.close()
    with pytest.raises(native.BlsGpuError):
        native.Context([n])  # past the device count: BGV_E_ARG
