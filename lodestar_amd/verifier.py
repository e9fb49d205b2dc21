"""BlsGpuVerifier — the IBlsVerifier drop-in over libblsgpu (Python host mirror).

Mirrors packages/beacon-node/src/chain/bls/ of the reference:

* ``IBlsVerifier`` / ``VerifySignatureOpts``              interface.ts:3-46
* ``BlsMultiThreadWorkerPool.verifySignatureSets``        multithread/index.ts:134-174
* job buffering (batchable sets held <= 100 ms)           multithread/index.ts:238-285, 406-412
* job packaging (``prepareWork``)                         multithread/index.ts:386-401
* ``close()`` rejecting queued jobs with QUEUE_ABORTED    multithread/index.ts:176-197
* ``chunkifyMaximizeChunkSize``                           multithread/utils.ts:4-19
* ``getAggregatedPubkeysCount``                           utils.ts:18-26

The per-job verification (batch, retry, error precedence) runs inside the
C-ABI library (bgv_verify, BGV_MODE_WORKER), i.e. on the GPU.  The host never
computes a verdict itself.  Names follow the reference in snake_case.
"""
from __future__ import annotations

import asyncio
import ctypes
import enum
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Union

from . import native

# multithread/index.ts:39,48,57 — kept as defaults; the GPU prefers bigger packages
MAX_SIGNATURE_SETS_PER_JOB = 128
MAX_BUFFERED_SIGS = 32
MAX_BUFFER_WAIT_MS = 100
# sets per device call (the reference sends <=128-sig packages to one worker)
MAX_SETS_PER_DEVICE_CALL = 16384


class SignatureSetType(enum.Enum):
    """state-transition/src/util/signatureSets.ts:5-8"""
    single = "single"
    aggregate = "aggregate"


# A public key is a validator index into the device cache (int) or 96 uncompressed bytes.
PublicKey = Union[int, bytes]


@dataclass
class ISignatureSet:
    """state-transition/src/util/signatureSets.ts:10-22"""
    type: SignatureSetType
    signing_root: bytes
    signature: bytes
    pubkey: Optional[PublicKey] = None
    pubkeys: List[PublicKey] = field(default_factory=list)


@dataclass
class VerifySignatureOpts:
    batchable: bool = False
    verify_on_main_thread: bool = False


class QueueError(Exception):
    """util/queue/errors.ts: QueueErrorCode.QUEUE_ABORTED"""

    def __init__(self, code: str = "QUEUE_ABORTED"):
        super().__init__(code)
        self.code = code


def chunkify_maximize_chunk_size(arr: Sequence, min_per_chunk: int) -> List[list]:
    """multithread/utils.ts:4-19"""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [list(arr)]
    per_chunk = -(-len(arr) // chunk_count)
    return [list(arr[i:i + per_chunk]) for i in range(0, len(arr), per_chunk)]


def get_aggregated_pubkeys_count(sets: Sequence[ISignatureSet]) -> int:
    """utils.ts:18-26"""
    return sum(len(s.pubkeys) for s in sets if s.type == SignatureSetType.aggregate)


def to_set_spec(s: ISignatureSet) -> native.SetSpec:
    """getAggregatedPubkey + serialisation (utils.ts:5-16, index.ts:158-163): the
    aggregation itself happens on the device."""
    if s.type == SignatureSetType.single:
        pks = [s.pubkey]
    elif s.type == SignatureSetType.aggregate:
        pks = list(s.pubkeys)
    else:
        raise ValueError("Unknown signature set type")
    if pks and all(isinstance(p, int) for p in pks):
        return native.SetSpec(s.signing_root, s.signature, pk_indices=pks)
    if all(isinstance(p, (bytes, bytearray)) for p in pks):
        return native.SetSpec(s.signing_root, s.signature, pk_bytes=[bytes(p) for p in pks])
    raise ValueError("mix of cached and uncached pubkeys in one set")


@dataclass
class _Job:
    sets: List[native.SetSpec]
    batchable: bool
    future: asyncio.Future
    added: float


class BlsGpuVerifier:
    """IBlsVerifier over the MI355X verifier (one bgv_ctx)."""

    def __init__(self, ctx: Optional[native.Context] = None, *, blsVerifyAllMultiThread: bool = False,
                 max_buffered_sigs: int = MAX_BUFFERED_SIGS, max_buffer_wait_ms: float = MAX_BUFFER_WAIT_MS,
                 max_sets_per_job: int = MAX_SIGNATURE_SETS_PER_JOB,
                 max_sets_per_device_call: int = MAX_SETS_PER_DEVICE_CALL):
        self.ctx = ctx or native.Context()
        self.verify_all_multi_thread = blsVerifyAllMultiThread
        self.max_buffered_sigs = max_buffered_sigs
        self.max_buffer_wait_ms = max_buffer_wait_ms
        self.max_sets_per_job = max_sets_per_job
        self.max_sets_per_device_call = max_sets_per_device_call
        self.jobs: List[_Job] = []
        self.buffered: Optional[dict] = None
        self.closed = False
        self.running = False
        self.metrics = {"aggregated_pubkeys": 0, "batch_retries": 0, "batch_sigs_success": 0,
                        "success_sets": 0, "error_sets": 0, "device_calls": 0, "device_ms": 0.0}

    # --- IBlsVerifier -------------------------------------------------------
    async def verify_signature_sets(self, sets: Sequence[ISignatureSet],
                                    opts: Optional[VerifySignatureOpts] = None) -> bool:
        opts = opts or VerifySignatureOpts()
        self.metrics["aggregated_pubkeys"] += get_aggregated_pubkeys_count(sets)
        if opts.verify_on_main_thread and not self.verify_all_multi_thread:
            # index.ts:138-151: synchronous, on the caller's thread
            code = self._verify_now([to_set_spec(s) for s in sets])
            return self._unwrap(code)
        results = await asyncio.gather(*[
            self._queue_bls_work([to_set_spec(s) for s in chunk], opts.batchable)
            for chunk in chunkify_maximize_chunk_size(list(sets), self.max_sets_per_job)
        ])
        if len(results) == 0:
            raise Exception("Empty results array")
        return all(r is True for r in results)

    async def is_valid_bls_aggregate(self, public_keys: Sequence[PublicKey], message: bytes,
                                     signature: bytes) -> bool:
        """Light-client sync-aggregate check, isValidBlsAggregate (light-client/src/validation.ts:
        152-176): PublicKey.aggregate(publicKeys), which throws on an empty list, then
        Signature.fromBytes(signature, undefined, true).verify(aggPubkey, message).  One
        non-batchable aggregate set on the device: an undecodable or non-G2 signature raises with
        its BLST code, an infinity aggregate verifies false (core verify of a one-set job)."""
        if len(public_keys) == 0:
            raise native.BlsGpuError(native.BGV_E_EMPTY_AGGREGATE)
        s = ISignatureSet(SignatureSetType.aggregate, signing_root=message, signature=signature,
                          pubkeys=list(public_keys))
        return await self.verify_signature_sets([s], VerifySignatureOpts(batchable=False))

    async def close(self):
        if self.buffered and self.buffered.get("timer"):
            self.buffered["timer"].cancel()
        for job in self.jobs + (self.buffered["jobs"] if self.buffered else []):
            if not job.future.done():
                job.future.set_exception(QueueError("QUEUE_ABORTED"))
        self.jobs = []
        self.buffered = None
        self.closed = True

    # --- internals ----------------------------------------------------------
    def _verify_now(self, sets) -> int:
        stats = native.BgvStats()
        codes = self.ctx.verify_jobs([(sets, False)], native.MODE_PER_JOB, stats)
        self._account(stats)
        return codes[0]

    @staticmethod
    def _unwrap(code: int) -> bool:
        if code < 0:
            raise native.BlsGpuError(-code)
        return code == 1

    def _account(self, stats: native.BgvStats):
        self.metrics["batch_retries"] += stats.batch_retries
        self.metrics["batch_sigs_success"] += stats.batch_sigs_success
        self.metrics["device_calls"] += 1
        self.metrics["device_ms"] += stats.device_ms

    async def _queue_bls_work(self, sets, batchable: bool) -> bool:
        if self.closed:
            raise QueueError("QUEUE_ABORTED")
        loop = asyncio.get_running_loop()
        job = _Job(sets, batchable, loop.create_future(), time.monotonic())
        if batchable:
            if self.buffered is None:
                self.buffered = {"jobs": [], "sig_count": 0,
                                 "timer": loop.call_later(self.max_buffer_wait_ms / 1e3, self._run_buffered_jobs)}
            self.buffered["jobs"].append(job)
            self.buffered["sig_count"] += len(sets)
            if self.buffered["sig_count"] > self.max_buffered_sigs:
                self.buffered["timer"].cancel()
                self._run_buffered_jobs()
        else:
            self.jobs.append(job)
            loop.call_soon(self._schedule_run)
        return await job.future

    def _run_buffered_jobs(self):
        if self.buffered is not None:
            self.jobs.extend(self.buffered["jobs"])
            self.buffered = None
            asyncio.get_running_loop().call_soon(self._schedule_run)

    def _schedule_run(self):
        if self.closed or self.running or not self.jobs:
            return
        self.running = True
        asyncio.ensure_future(self._run_job())

    def _prepare_work(self) -> List[_Job]:
        """index.ts:386-401 with a GPU-sized package"""
        out, total = [], 0
        while self.jobs and total < self.max_sets_per_device_call:
            job = self.jobs.pop(0)
            out.append(job)
            total += len(job.sets)
        return out

    async def _run_job(self):
        try:
            while self.jobs and not self.closed:
                jobs = self._prepare_work()
                loop = asyncio.get_running_loop()
                try:
                    stats = native.BgvStats()
                    codes = await loop.run_in_executor(
                        None, lambda: self.ctx.verify_jobs([(j.sets, j.batchable) for j in jobs],
                                                           native.MODE_WORKER, stats))
                    self._account(stats)
                except Exception as e:  # device failure: reject, never a verdict
                    for j in jobs:
                        if not j.future.done():
                            j.future.set_exception(e)
                    continue
                for j, code in zip(jobs, codes):
                    if j.future.done():
                        continue
                    if code < 0:
                        self.metrics["error_sets"] += len(j.sets)
                        j.future.set_exception(native.BlsGpuError(-code))
                    else:
                        self.metrics["success_sets"] += len(j.sets)
                        j.future.set_result(code == 1)
        finally:
            self.running = False
            if self.jobs and not self.closed:
                asyncio.get_running_loop().call_soon(self._schedule_run)


class BlsGpuSingleThreadVerifier:
    """BlsSingleThreadVerifier equivalent (singleThread.ts:7-40): every call verified
    at once as one job; opts ignored."""

    def __init__(self, ctx: Optional[native.Context] = None):
        self.ctx = ctx or native.Context()

    async def verify_signature_sets(self, sets: Sequence[ISignatureSet], opts=None) -> bool:
        codes = self.ctx.verify_jobs([([to_set_spec(s) for s in sets], False)], native.MODE_PER_JOB)
        return BlsGpuVerifier._unwrap(codes[0])

    async def close(self):
        pass


__all__ = ["BlsGpuVerifier", "BlsGpuSingleThreadVerifier", "ISignatureSet", "SignatureSetType",
           "VerifySignatureOpts", "QueueError", "chunkify_maximize_chunk_size", "get_aggregated_pubkeys_count",
           "ctypes"]
