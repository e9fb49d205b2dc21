"""Multi-process path on the CPU with gloo, world size 2.

* shard_bounds: job-boundary partition balanced by set count;
* ShardedVerify: each rank verifies its shard, verdicts all-gathered — checked on the
  golden verdict vectors, with the C++ CPU restatement standing in for the device as the
  per-rank verify function (test harness only; tests/test_gpu_distributed.py runs the same
  class over native.Context on the GPU);
* a rank whose device call fails: every rank joins the collective and raises (no hang,
  no verdict);
* verify_one_job: the Fp12-partial protocol's code combination in set order (signature
  errors first, then pubkey conditions, then the verdict) with stand-in partial functions;
* bench.py's Barrier: barrier + max-over-ranks of the timed region.
"""
import json
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from lodestar_amd.shard import ShardedVerify, shard_bounds  # noqa: E402

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


def _fault_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lodestar_amd import native

        def verify_fn(js):
            if rank == 1:
                raise native.DeviceError("BGV_E_DEVICE: HIP device error")
            return [1] * len(js)

        jobs = [([("s", i)], True) for i in range(6)]
        try:
            got = ShardedVerify(verify_fn, dist)(jobs)
            q.put((rank, "returned %r" % got))
        except native.DeviceError:
            q.put((rank, "raised"))
        # one job: a failing partial on rank 0 raises everywhere too
        def partial_fn(sets):
            if rank == 0:
                raise native.DeviceError("BGV_E_DEVICE: HIP device error")
            return ONE, 0, 0
        try:
            code = ShardedVerify(None, dist, partial_fn=partial_fn, final_fn=lambda p: True).verify_one_job(
                [("s", i) for i in range(4)])
            q.put((rank, "one-job returned %r" % code))
        except native.DeviceError:
            q.put((rank, "one-job raised"))
    finally:
        dist.destroy_process_group()


ONE = bytes(47) + b"\x01" + bytes(528)
BAD = b"\x02" * 576


def _one_job_worker(rank, world, port, q):
    """Stand-in partials: a set is (valid, sig_code, pk_code); the shard's partial is ONE
    iff every set is valid, and final_fn accepts iff every partial is ONE."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def partial_fn(sets):
            sc = next((s for _, s, _ in sets if s), 0)
            pc = next((p for _, _, p in sets if p), 0)
            return (ONE if all(v for v, _, _ in sets) else BAD), sc, pc

        sv = ShardedVerify(None, dist, partial_fn=partial_fn, final_fn=lambda ps: all(p == ONE for p in ps))
        ok = [(1, 0, 0)] * 8
        cases = {
            "valid": (ok, 1),
            "invalid_on_rank1": (ok[:6] + [(0, 0, 0)] + ok[7:], 0),
            # signature errors win over pubkey conditions, the first in set order wins
            "sig_err_rank1_pk_err_rank0": ([(1, 0, -2)] + ok[1:5] + [(1, -1, 0)] + ok[6:], -1),
            "two_sig_errs": ([(1, 0, 0), (1, -3, 0)] + ok[2:6] + [(1, -8, 0)] + ok[7:], -3),
            "pk_infinity": (ok[:5] + [(1, 0, 1)] + ok[6:], -6),
            "pk_infinity_single_set": ([(1, 0, 1)], 0),
            "empty": ([], -21),
        }
        q.put((rank, {k: sv.verify_one_job(v[0]) == v[1] for k, v in cases.items()}))
    finally:
        dist.destroy_process_group()


def _fast_path_worker(rank, world, port, q):
    """fast_path=True with stand-in partials (as _one_job_worker): an empty job rejects with
    BGV_E_EMPTY_SET (-21) as on the per-job path, whether the combined check passes or a
    shard falls back to verify_fn."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def partial_fn(sets):
            return (ONE if all(v for v, _, _ in sets) else BAD), 0, 0

        def verify_fn(js):
            return [(-21 if not ss else (1 if all(v for v, _, _ in ss) else 0)) for ss, _ in js]

        sv = ShardedVerify(verify_fn, dist, partial_fn=partial_fn,
                           final_fn=lambda ps: all(p == ONE for p in ps), fast_path=True)
        good = ([(1, 0, 0)], True)
        bad = ([(0, 0, 0)], True)
        empty = ([], True)
        out = {
            "clean_with_empty": sv([good, empty, good, good, empty, good]) == [1, -21, 1, 1, -21, 1],
            "failing_with_empty": sv([good, empty, good, bad, empty, good]) == [1, -21, 1, 0, -21, 1],
            "only_empty": sv([empty, empty]) == [-21, -21],
        }
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_fast_path_empty_job():
    for rank, ok in _spawn(_fast_path_worker):
        assert all(ok.values()), (rank, ok)


def _spawn(target, world=2):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world * (2 if target is _fault_worker else 1)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


def test_device_error_on_one_rank_raises_everywhere():
    res = _spawn(_fault_worker)
    assert [r[1] for r in res] == ["one-job raised", "raised", "one-job raised", "raised"], res


def test_one_job_code_combination():
    for rank, ok in _spawn(_one_job_worker):
        assert all(ok.values()), (rank, ok)


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
