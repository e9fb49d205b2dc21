"""Sharding verification over one process per GPU.

The reference has no multi-device path: BlsMultiThreadWorkerPool spreads a call's jobs over
worker threads (packages/beacon-node/src/chain/bls/multithread/index.ts:153-166, 199-233).
Here a call spreads over GPUs, one process each, in two ways:

* Many jobs (gossip, config 4 mode (i)): jobs are independent, so `ShardedVerify.__call__`
  splits them at job boundaries (`shard_bounds`, balanced by set count), every rank verifies
  its shard on its own device (`native.Context.verify_jobs`, per-job batch + retry inside the
  library) and the per-job codes are all-gathered (4 B per job).
  With `fast_path=True` each rank first reduces its whole shard to one Fp12 Miller-loop
  product (bgv_verify_partial); the partials are gathered and ONE final exponentiation
  decides the call.  If it passes, every job is valid.  Otherwise each rank checks its own
  partial (one final exponentiation) and only failing shards re-verify per job (SURVEY
  §8(e), "Retry").
* One job (a block range, config 4 mode (ii), the config-5 epoch sweep as one call):
  `ShardedVerify.verify_one_job` splits the job's sets over ranks; each rank computes its
  shard's partial product e(r_i pk_i, H(m_i)) ... e(-G1, sum r_i sig_i) (576 B), the partials
  are all-gathered over the process group (RCCL over xGMI with the "nccl" backend, gloo on
  the CPU), and every rank multiplies them and runs the single final exponentiation
  (bgv_final_verify), so all ranks return the same code without a second collective.

Error precedence follows job_precheck (bgv_api.cpp) / maybeBatch.ts:16-39 over the whole
job: the first undecodable signature in set order (rank order = set order), else the first
pubkey condition (infinity aggregate: BLST_PK_IS_INFINITY for >= 2 sets, false for one set).
A device error on any rank never becomes a verdict: every rank joins the collective with
an error marker and then raises.
"""
from typing import Callable, List, Optional, Sequence, Tuple

BGV_E_DEVICE = 30
BGV_E_EMPTY_SET = 21
BLST_PK_IS_INFINITY = 6
ONE_FP12 = bytes(47) + b"\x01" + bytes(528)  # canonical bytes of 1 in GT's Fp12


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
    """Verification of calls split over the ranks of a process group.

    verify_fn(jobs) -> list of int codes (1, 0, -error), one per job (the device path,
    native.Context.verify_jobs).  partial_fn(sets) -> (576-byte partial, sig_code, pk_code)
    and final_fn(partials) -> bool are native.Context.verify_partial / final_verify.
    """

    def __init__(self, verify_fn: Callable[[list], List[int]], dist, group=None,
                 partial_fn: Optional[Callable] = None, final_fn: Optional[Callable] = None,
                 fast_path: bool = False):
        self.verify_fn = verify_fn
        self.partial_fn = partial_fn
        self.final_fn = final_fn
        self.fast_path = fast_path
        self.dist = dist
        self.group = group

    # --- transport ------------------------------------------------------------
    def _device(self):
        import torch
        if self.dist.get_backend(self.group) == "nccl":  # RCCL over xGMI on ROCm
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _all_gather_bytes(self, payload: bytes, width: int) -> List[bytes]:
        import torch
        dev = self._device()
        buf = torch.zeros(width, dtype=torch.uint8)
        if payload:
            buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
        buf = buf.to(dev)
        world = self.dist.get_world_size(self.group)
        parts = [torch.zeros(width, dtype=torch.uint8, device=dev) for _ in range(world)]
        self.dist.all_gather(parts, buf, group=self.group)
        return [bytes(p.cpu().numpy().tobytes()) for p in parts]

    def _gather_codes(self, local: List[int], width: int) -> List[List[int]]:
        import numpy as np
        raw = np.zeros(width + 1, dtype=np.int32)
        raw[0] = len(local)
        raw[1:1 + len(local)] = local
        out = []
        for b in self._all_gather_bytes(raw.tobytes(), 4 * (width + 1)):
            a = np.frombuffer(b, dtype=np.int32)
            out.append([int(x) for x in a[1:1 + a[0]]])
        return out

    # --- many jobs --------------------------------------------------------------
    def __call__(self, jobs: list) -> List[int]:
        world = self.dist.get_world_size(self.group)
        rank = self.dist.get_rank(self.group)
        bounds = shard_bounds([len(sets) for sets, _ in jobs], world)
        lo, hi = bounds[rank]
        mine = jobs[lo:hi]
        err = None
        local: Optional[List[int]] = None
        if self.fast_path and self.partial_fn is not None:
            local, err = self._fast(mine)
        if local is None and err is None:
            try:
                local = list(self.verify_fn(mine)) if mine else []
                if len(local) != len(mine):
                    raise RuntimeError("verify_fn returned %d codes for %d jobs" % (len(local), len(mine)))
            except Exception as e:  # noqa: BLE001 -- joined the collective below, then re-raised
                err = e
        if err is not None:
            local = [-BGV_E_DEVICE] * len(mine)
        width = max(h - l for l, h in bounds)
        parts = self._gather_codes(local, width)
        if err is not None:
            raise err
        out: List[int] = []
        for p in parts:
            out.extend(p)
        if any(c == -BGV_E_DEVICE for c in out):
            from .native import DeviceError
            raise DeviceError("BGV_E_DEVICE on another rank")
        return out

    def _fast(self, mine):
        """Whole-call partial products: (codes or None, error).  None codes = verify per job.
        A job with no sets rejects with BGV_E_EMPTY_SET ("Empty signature set",
        maybeBatch.ts:29-31) as on the per-job path; it adds nothing to the partial."""
        sets = [s for ss, _ in mine for s in ss]
        try:
            partial, sc, pc = self.partial_fn(sets) if sets else (ONE_FP12, 0, 0)
            ok = 1
        except Exception as e:  # noqa: BLE001
            partial, sc, pc, ok = ONE_FP12, 0, 0, 0
            err = e
        else:
            err = None
        import struct
        parts = self._all_gather_bytes(partial + struct.pack("<iii", sc, pc, ok), 588)
        if err is not None:
            return None, err
        if not all(struct.unpack("<iii", p[576:])[2] for p in parts):
            from .native import DeviceError
            return None, DeviceError("BGV_E_DEVICE on another rank")
        clean = all(struct.unpack("<iii", p[576:])[:2] == (0, 0) for p in parts)
        ok_codes = [1 if ss else -BGV_E_EMPTY_SET for ss, _ in mine]
        if clean and self.final_fn([p[:576] for p in parts]):
            return ok_codes, None  # one final exponentiation for the whole call
        if sc == 0 and pc == 0 and self.final_fn([partial]):
            return ok_codes, None  # this shard is clean: only failing shards retry
        return None, None

    # --- one job --------------------------------------------------------------------
    def verify_one_job(self, sets: list) -> int:
        """One job's sets split over the ranks; Fp12 partials gathered, one final
        exponentiation.  Returns the job's code (1, 0 or -BLST error) on every rank."""
        world = self.dist.get_world_size(self.group)
        rank = self.dist.get_rank(self.group)
        if not sets:
            return -BGV_E_EMPTY_SET  # "Empty signature set" (maybeBatch.ts:29-31)
        lo, hi = shard_bounds([1] * len(sets), world)[rank]
        return self.one_job_from_shard(lambda: self.partial_fn(sets[lo:hi]) if hi > lo else (ONE_FP12, 0, 0),
                                       len(sets))

    def one_job_from_shard(self, shard_partial: Callable[[], tuple], nsets: int) -> int:
        """The collective half of verify_one_job: this rank's shard_partial() ->
        (576-B partial, sig_code, pk_code) is all-gathered (RCCL with the nccl backend) and
        every rank runs the one final exponentiation.  Callers that hold their shard in
        another form (native.PackedSingleSets: the config-5 sweep) use this directly."""
        import struct
        err = None
        try:
            partial, sc, pc = shard_partial()
            ok = 1
        except Exception as e:  # noqa: BLE001 -- joined the collective below, then re-raised
            partial, sc, pc, ok, err = ONE_FP12, 0, 0, 0, e
        parts = self._all_gather_bytes(partial + struct.pack("<iii", sc, pc, ok), 588)
        if err is not None:
            raise err
        codes = [struct.unpack("<iii", p[576:]) for p in parts]
        if not all(c[2] for c in codes):
            from .native import DeviceError
            raise DeviceError("BGV_E_DEVICE on another rank")
        for s, _, _ in codes:  # first undecodable signature in set order
            if s:
                return s
        for _, p, _ in codes:  # then the first pubkey condition
            if p == 1:
                return -BLST_PK_IS_INFINITY if nsets >= 2 else 0
            if p:
                return p
        return 1 if self.final_fn([p[:576] for p in parts]) else 0
