"""Sharding a verify call over one process per GPU.

Signature sets are independent and every device group ends in its own final
exponentiation, so a call splits over ranks at job boundaries with no
data-path exchange.  The only collective is the gather of the per-job verdict
codes (4 bytes per job) so that every rank can answer the caller; the
reference has no multi-device path (BlsMultiThreadWorkerPool spreads jobs over
worker threads, multithread/index.ts:290-381), and this is its process-level
analogue.

`shard_bounds` balances ranks by set count (jobs are never split: a job's
verdict is one boolean, multithread/types.ts:14-17).  `ShardedVerify` runs the
local slice through a verify function (the device path, `native.Context.verify_jobs`)
and all-gathers the codes over the given process group (gloo or RCCL).
"""
from typing import Callable, List, Sequence, Tuple


def shard_bounds(job_sizes: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) job ranges per rank, cut where the running set count
    crosses k * total / world.  Every rank gets a range (possibly empty)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    total = sum(job_sizes)
    bounds, lo, acc, r = [], 0, 0, 1
    for j, n in enumerate(job_sizes):
        acc += n
        while r < world and acc * world >= r * total and total > 0:
            bounds.append((lo, j + 1))
            lo = j + 1
            r += 1
    while len(bounds) < world - 1:
        bounds.append((lo, lo))
    bounds.append((lo, len(job_sizes)))
    return bounds


class ShardedVerify:
    """verify(jobs) on this rank's shard, then all-gather the verdicts.

    verify_fn(jobs) -> list of int codes (1, 0, -error), one per job.
    """

    def __init__(self, verify_fn: Callable[[list], List[int]], dist, group=None):
        self.verify_fn = verify_fn
        self.dist = dist
        self.group = group

    def __call__(self, jobs: list) -> List[int]:
        import torch
        world = self.dist.get_world_size(self.group)
        rank = self.dist.get_rank(self.group)
        bounds = shard_bounds([len(sets) for sets, _ in jobs], world)
        lo, hi = bounds[rank]
        local = self.verify_fn(jobs[lo:hi]) if hi > lo else []
        if len(local) != hi - lo:
            raise RuntimeError("verify_fn returned %d codes for %d jobs" % (len(local), hi - lo))
        width = max(h - l for l, h in bounds)
        buf = torch.zeros(width, dtype=torch.int32)
        if local:
            buf[:len(local)] = torch.tensor(local, dtype=torch.int32)
        parts = [torch.zeros(width, dtype=torch.int32) for _ in range(world)]
        self.dist.all_gather(parts, buf, group=self.group)
        out: List[int] = []
        for (l, h), p in zip(bounds, parts):
            out.extend(int(x) for x in p[:h - l])
        return out
