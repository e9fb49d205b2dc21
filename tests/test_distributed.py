"""Multi-process path on the CPU with gloo, world size 2.

* shard_bounds: job-boundary partition balanced by set count;
* ShardedVerify: each rank verifies its shard, verdicts all-gathered — checked on the
  golden verdict vectors, with the C++ CPU restatement standing in for the device as the
  per-rank verify function (test harness only; on the GPU box the same class wraps
  native.Context.verify_jobs);
* bench.py's Barrier: barrier + max-over-ranks of the timed region.
"""
import json
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from lodestar_amd.shard import ShardedVerify, shard_bounds

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_shard_bounds():
    assert shard_bounds([1, 1, 1, 1], 2) == [(0, 2), (2, 4)]
    assert shard_bounds([128, 1, 1, 1], 2) == [(0, 1), (1, 4)]
    assert shard_bounds([], 3) == [(0, 0), (0, 0), (0, 0)]
    assert sum(h - l for l, h in shard_bounds([5], 4)) == 1
    for sizes in ([3, 1, 4, 1, 5, 9, 2, 6], [1] * 17, [64] * 3 + [1] * 40):
        for world in (1, 2, 3, 8):
            b = shard_bounds(sizes, world)
            assert len(b) == world
            assert b[0][0] == 0 and b[-1][1] == len(sizes)
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            loads = [sum(sizes[l:h]) for l, h in b]
            assert max(loads) <= sum(sizes) / world + max(sizes)


def _golden_jobs():
    from oracle import bls12381 as o
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
    return jobs, exp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.cpu import blscpu
        jobs, exp = _golden_jobs()
        seen = []

        def verify_fn(js):
            seen.append(len(js))
            return blscpu.verify_jobs(js, 0, threads=1)

        got = ShardedVerify(verify_fn, dist)(jobs)
        import bench
        b = bench.Barrier.__new__(bench.Barrier)
        b.world, b.dist = world, dist
        b()
        mx = b.max(float(rank + 1))
        q.put((rank, got == exp, seen, mx))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_verify_gloo_world2():
    from oracle.cpu import blscpu
    blscpu.lib()  # build before forking
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for rank, ok, seen, mx in res:
        assert ok, "rank %d gathered verdicts differ from the golden codes" % rank
        assert mx == float(world)
    assert sum(sum(s) for _, _, s, _ in res) == len(_golden_jobs()[1])
    assert all(s for _, _, s, _ in res), "every rank verifies a non-empty shard"


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
