"""ctypes binding of libblsgpu.so (include/blsgpu.h).

This is the Python side of the drop-in boundary; the N-API addon described in
INTEGRATION.md binds the same symbols for Node.  There is no CPU fallback:
loading fails loudly when the HIP library is missing or no device is present.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import List, Optional, Sequence

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BLSGPU_LIB", os.path.join(HERE, "libblsgpu.so"))

# status codes (include/blsgpu.h)
BGV_OK = 0
BLST_BAD_ENCODING = 1
BLST_POINT_NOT_ON_CURVE = 2
BLST_POINT_NOT_IN_GROUP = 3
BLST_PK_IS_INFINITY = 6
BLST_INVALID_SIZE = 8
BGV_E_EMPTY_AGGREGATE = 20
BGV_E_EMPTY_SET = 21
BGV_E_BAD_INDEX = 22
BGV_E_ARG = 23
BGV_E_DEVICE = 30
BGV_E_CLOSED = 32

MODE_WORKER = 0
MODE_PER_JOB = 1
PATH_BULK = 1
PATH_LATENCY = 2
PK_COMPRESSED = 48
PK_UNCOMPRESSED = 96

EXPORTED_SYMBOLS = [
    "bgv_init", "bgv_close", "bgv_destroy", "bgv_pubkeys_put", "bgv_pubkeys_count", "bgv_verify",
    "bgv_verify_async", "bgv_aggregate_pubkeys", "bgv_hash_to_g2", "bgv_keygen", "bgv_sign",
    "bgv_set_rng_seed", "bgv_strerror", "bgv_device_count", "bgv_profile",
    "bgv_pubkeys_validate", "bgv_aggregate_signatures", "bgv_deposits_verify", "bgv_set_batching",
    "bgv_verify_partial", "bgv_final_verify", "bgv_debug_prepare", "bgv_debug_uniform", "bgv_set_split",
]


class BgvSet(ctypes.Structure):
    _fields_ = [
        ("n_pk", ctypes.c_uint32),
        ("sig_len", ctypes.c_uint32),
        ("pk_indices", ctypes.c_void_p),
        ("pk_bytes", ctypes.c_void_p),
        ("msg", ctypes.c_void_p),
        ("sig", ctypes.c_void_p),
    ]


class BgvJob(ctypes.Structure):
    _fields_ = [("first_set", ctypes.c_uint32), ("n_sets", ctypes.c_uint32), ("batchable", ctypes.c_uint32)]


class BgvStats(ctypes.Structure):
    _fields_ = [
        ("batch_retries", ctypes.c_uint64),
        ("batch_sigs_success", ctypes.c_uint64),
        ("device_groups", ctypes.c_uint64),
        ("sets_verified", ctypes.c_uint64),
        ("device_ms", ctypes.c_double),
        ("wall_ms", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int)

_lib = None
_lib_lock = threading.Lock()


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libblsgpu.so; raises if it is missing (no fallback path exists)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError("libblsgpu.so not built (%s): run `python -m lodestar_amd.build`" % path)
        lib = ctypes.CDLL(path)
        P, U32, SZ, I32, U64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int32, ctypes.c_uint64
        sig = {
            "bgv_init": ([P, ctypes.c_int, P], ctypes.c_int),
            "bgv_close": ([P], ctypes.c_int),
            "bgv_destroy": ([P], ctypes.c_int),
            "bgv_pubkeys_put": ([P, U32, P, SZ, ctypes.c_int], ctypes.c_int),
            "bgv_pubkeys_count": ([P], SZ),
            "bgv_verify": ([P, P, SZ, P, SZ, ctypes.c_int, P, P], ctypes.c_int),
            "bgv_verify_async": ([P, P, SZ, P, SZ, ctypes.c_int, P, P, DONE_FN, P], ctypes.c_int),
            "bgv_aggregate_pubkeys": ([P, P, SZ, P], ctypes.c_int),
            "bgv_hash_to_g2": ([P, P, P, SZ, P], ctypes.c_int),
            "bgv_keygen": ([P, P, SZ, ctypes.c_int64, P], ctypes.c_int),
            "bgv_sign": ([P, P, P, SZ, P], ctypes.c_int),
            "bgv_set_rng_seed": ([P, U64], ctypes.c_int),
            "bgv_set_batching": ([P, U32, U32, U32], ctypes.c_int),
            "bgv_set_split": ([P, U32], ctypes.c_int),
            "bgv_verify_partial": ([P, P, SZ, P, P], ctypes.c_int),
            "bgv_final_verify": ([P, P, SZ, P], ctypes.c_int),
            "bgv_debug_prepare": ([P, P, SZ, ctypes.c_int, U64, P, P, P], ctypes.c_int),
            "bgv_debug_uniform": ([P, P, SZ, U64, P, P, SZ, P, P, P], ctypes.c_int),
            "bgv_strerror": ([ctypes.c_int], ctypes.c_char_p),
            "bgv_device_count": ([], ctypes.c_int),
            "bgv_profile": ([P, ctypes.c_int, P, P, ctypes.c_int, P], ctypes.c_int),
            "bgv_pubkeys_validate": ([P, P, SZ, P, P], ctypes.c_int),
            "bgv_aggregate_signatures": ([P, P, P, P, SZ, P, P], ctypes.c_int),
            "bgv_deposits_verify": ([P, P, P, P, SZ, P], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            if name in ("bgv_debug_prepare", "bgv_debug_uniform", "bgv_set_split") and path != os.path.join(HERE, "libblsgpu.so") and \
                    not hasattr(lib, name):
                continue  # parity hook absent from an older A/B build (tools/gpu/ab.sh)
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        del I32
        _lib = lib
        return lib


def strerror(code: int) -> str:
    return load().bgv_strerror(int(code)).decode()


class BlsGpuError(Exception):
    """Rejection carrying a BLST-style code; str() contains the code name
    (e.g. "BLST_INVALID_SIZE"), like the reference worker's Error(message)."""

    def __init__(self, code: int):
        self.code = abs(int(code))
        super().__init__(strerror(self.code))


class DeviceError(RuntimeError):
    pass


def _check(rc: int):
    if rc < 0:
        if -rc == BGV_E_DEVICE:
            raise DeviceError(strerror(rc))
        raise BlsGpuError(-rc)
    return rc


def _buf(b: bytes):
    return ctypes.create_string_buffer(bytes(b), len(b)) if len(b) else ctypes.create_string_buffer(1)


class Context:
    """One bgv_ctx (device-resident pubkey cache + per-call buffers)."""

    def __init__(self, devices: Optional[Sequence[int]] = None):
        self.lib = load()
        if self.lib.bgv_device_count() <= 0:
            raise DeviceError("no HIP device visible to libblsgpu")
        self._h = ctypes.c_void_p()
        devs = list(devices or [])
        arr = (ctypes.c_int * max(1, len(devs)))(*devs) if devs else None
        _check(self.lib.bgv_init(arr, len(devs), ctypes.byref(self._h)))

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            self.lib.bgv_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_batching(self, max_batch_slots: int = 0, coalesce_us: int = 0xFFFFFFFF,
                     idle_coalesce_us: int = 0xFFFFFFFF):
        """Super-batch geometry (bgv_set_batching); 0 / 0xFFFFFFFF leave a value unchanged."""
        _check(self.lib.bgv_set_batching(self._h, max_batch_slots, coalesce_us, idle_coalesce_us))

    def set_split(self, min_sets: int):
        """Calls of at least min_sets sets spread over the context's devices (bgv_set_split;
        0 disables)."""
        _check(self.lib.bgv_set_split(self._h, min_sets))

    def verify_packed_one_job(self, packed: "PackedSingleSets", mode: int = MODE_PER_JOB,
                              stats: Optional[BgvStats] = None) -> int:
        """One job over all of a PackedSingleSets' sets (bgv_verify): its code."""
        job = BgvJob(0, packed.nsets, 0)
        out = (ctypes.c_int32 * 1)()
        _check(self.lib.bgv_verify(self._h, ctypes.byref(job), 1, packed.ptr(), packed.nsets, mode, out,
                                   ctypes.byref(stats) if stats is not None else None))
        return out[0]

    def set_rng_seed(self, seed: int):
        _check(self.lib.bgv_set_rng_seed(self._h, seed))

    def profile(self, enable: int = -1):
        """Per-kernel accumulated device ms since the last reset: ({name: ms}, launches);
        enable 1/0 resets and switches event recording on/off, -1 only reads."""
        n = 16
        ms = (ctypes.c_double * n)()
        names = (ctypes.c_char_p * n)()
        launches = ctypes.c_uint64()
        k = _check(self.lib.bgv_profile(self._h, enable, ms, names, n, ctypes.byref(launches)))
        return {names[i].decode(): ms[i] for i in range(k)}, launches.value

    # --- pubkey cache -------------------------------------------------------
    def pubkeys_put(self, first_index: int, keys: bytes, fmt: int = PK_COMPRESSED):
        n = len(keys) // fmt
        assert n * fmt == len(keys)
        _check(self.lib.bgv_pubkeys_put(self._h, first_index, _buf(keys), n, fmt))

    def pubkeys_count(self) -> int:
        return self.lib.bgv_pubkeys_count(self._h)

    def keygen(self, sks: bytes, cache_first: int = -1, want_pubkeys: bool = True) -> bytes:
        n = len(sks) // 32
        out = ctypes.create_string_buffer(48 * n) if want_pubkeys else None
        _check(self.lib.bgv_keygen(self._h, _buf(sks), n, cache_first, out))
        return out.raw if want_pubkeys else b""

    def sign(self, sks: bytes, msgs: bytes) -> bytes:
        n = len(sks) // 32
        assert len(msgs) == 32 * n
        out = ctypes.create_string_buffer(96 * n)
        _check(self.lib.bgv_sign(self._h, _buf(sks), _buf(msgs), n, out))
        return out.raw

    # --- parity hooks -------------------------------------------------------
    def aggregate_pubkeys(self, indices: Sequence[int]) -> bytes:
        arr = (ctypes.c_uint32 * max(1, len(indices)))(*indices)
        out = ctypes.create_string_buffer(96)
        _check(self.lib.bgv_aggregate_pubkeys(self._h, arr, len(indices), out))
        return out.raw

    def hash_to_g2(self, msgs: Sequence[bytes]) -> List[bytes]:
        lens = (ctypes.c_uint32 * max(1, len(msgs)))(*[len(m) for m in msgs])
        out = ctypes.create_string_buffer(192 * len(msgs))
        _check(self.lib.bgv_hash_to_g2(self._h, _buf(b"".join(msgs)), lens, len(msgs), out))
        return [out.raw[192 * i:192 * i + 192] for i in range(len(msgs))]

    # --- deposit keys, op-pool aggregation, deposit signatures ----
    def pubkeys_validate(self, keys48: Sequence[bytes]):
        """PublicKey.fromBytes(pk, affine, validate=true) per key -> (codes, uncompressed)."""
        n = len(keys48)
        st = (ctypes.c_int32 * max(1, n))()
        out = ctypes.create_string_buffer(96 * max(1, n))
        _check(self.lib.bgv_pubkeys_validate(self._h, _buf(b"".join(keys48)), n, st, out))
        return list(st[:n]), [out.raw[96 * i:96 * i + 96] for i in range(n)]

    def aggregate_signatures(self, aggregates: Sequence[Sequence[bytes]]):
        """Signature.aggregate over each list of signatures -> [(code, compressed96)]."""
        sigs = [s for agg in aggregates for s in agg]
        counts = (ctypes.c_uint32 * max(1, len(aggregates)))(*[len(a) for a in aggregates])
        lens = (ctypes.c_uint32 * max(1, len(sigs)))(*[len(x) for x in sigs])
        raw = b"".join(bytes(x[:96]).ljust(96, b"\0") for x in sigs)
        out = ctypes.create_string_buffer(96 * max(1, len(aggregates)))
        st = (ctypes.c_int32 * max(1, len(aggregates)))()
        _check(self.lib.bgv_aggregate_signatures(self._h, _buf(raw), lens, counts, len(aggregates), out, st))
        return [(st[a], out.raw[96 * a:96 * a + 96]) for a in range(len(aggregates))]

    def deposits_verify(self, keys48: Sequence[bytes], msgs: Sequence[bytes], sigs: Sequence[bytes]) -> List[int]:
        n = len(keys48)
        assert len(msgs) == n and len(sigs) == n and all(len(x) == 96 for x in sigs)
        out = (ctypes.c_int32 * max(1, n))()
        _check(self.lib.bgv_deposits_verify(self._h, _buf(b"".join(keys48)), _buf(b"".join(msgs)),
                                            _buf(b"".join(sigs)), n, out))
        return list(out[:n])

    # --- verification -------------------------------------------------------
    def verify_partial(self, sets) -> tuple:
        """One job's shard (list of SetSpec) -> (576-byte Miller-loop product, sig_code, pk_code)
        (bgv_verify_partial)."""
        packed = PackedCall([(list(sets), False)])
        out = ctypes.create_string_buffer(576)
        codes = (ctypes.c_int32 * 2)()
        _check(self.lib.bgv_verify_partial(self._h, packed.sets, packed.nsets, out, codes))
        return out.raw, codes[0], codes[1]

    def verify_partial_packed(self, packed: "PackedSingleSets", lo: int, hi: int) -> tuple:
        """verify_partial over sets [lo, hi) of a PackedSingleSets (no per-set objects)."""
        if not 0 <= lo <= hi <= packed.nsets:
            raise ValueError("shard bounds out of range")
        out = ctypes.create_string_buffer(576)
        codes = (ctypes.c_int32 * 2)()
        _check(self.lib.bgv_verify_partial(self._h, packed.ptr(lo), hi - lo, out, codes))
        return out.raw, codes[0], codes[1]

    def debug_prepare(self, sets, path: int, seed: int = 1):
        """bgv_debug_prepare (parity hook): per set (H(m) 192 B, f 576 B, sig status,
        pk status) from the bulk (PATH_BULK) or latency (PATH_LATENCY) kernels."""
        packed = PackedCall([(list(sets), False)])
        n = packed.nsets
        h = ctypes.create_string_buffer(192 * max(1, n))
        f = ctypes.create_string_buffer(576 * max(1, n))
        st = (ctypes.c_int32 * max(2, 2 * n))()
        _check(self.lib.bgv_debug_prepare(self._h, packed.sets, n, path, seed, h, f, st))
        return [(h.raw[192 * i:192 * i + 192], f.raw[576 * i:576 * i + 576], st[2 * i], st[2 * i + 1])
                for i in range(n)]

    def debug_uniform(self, sets, seed: int, tests=()):
        """bgv_debug_uniform (parity hook): one uniform group of the sets (one signing root) and
        retry tests over it, tests = [(slot mask, weighted)].  Returns (MillerLoop(sum r_i pk_i, H),
        [(test's pubkey-sum pair, test's signature pair)]), 576 B each."""
        packed = PackedCall([(list(sets), False)])
        n, nt = packed.nsets, len(tests)
        masks = (ctypes.c_uint64 * max(1, nt))(*[m for m, _ in tests])
        wts = (ctypes.c_uint32 * max(1, nt))(*[1 if w else 0 for _, w in tests])
        first = ctypes.create_string_buffer(576)
        pk = ctypes.create_string_buffer(576 * max(1, nt))
        sig = ctypes.create_string_buffer(576 * max(1, nt))
        _check(self.lib.bgv_debug_uniform(self._h, packed.sets, n, seed, masks, wts, nt, first, pk, sig))
        return first.raw, [(pk.raw[576 * t:576 * t + 576], sig.raw[576 * t:576 * t + 576]) for t in range(nt)]

    def final_verify(self, partials: Sequence[bytes]) -> bool:
        """Product of serialized partials and one final exponentiation == 1 (bgv_final_verify)."""
        v = ctypes.c_int32()
        _check(self.lib.bgv_final_verify(self._h, _buf(b"".join(partials)), len(partials), ctypes.byref(v)))
        return v.value == 1

    def verify_jobs(self, jobs, mode: int = MODE_WORKER, stats: Optional[BgvStats] = None) -> List[int]:
        """jobs: list of (sets, batchable) with sets = list of SetSpec.  Returns the
        per-job codes (1 valid, 0 invalid, -code error)."""
        packed = PackedCall(jobs)
        out = (ctypes.c_int32 * max(1, len(jobs)))()
        rc = self.lib.bgv_verify(self._h, packed.jobs, len(jobs), packed.sets, packed.nsets, mode, out,
                                 ctypes.byref(stats) if stats is not None else None)
        _check(rc)
        return list(out[:len(jobs)])


class SetSpec:
    """One ISignatureSet in C-ABI terms: pubkeys by cache index or 96-B bytes."""

    __slots__ = ("pk_indices", "pk_bytes", "msg", "sig")

    def __init__(self, msg: bytes, sig: bytes, pk_indices: Optional[Sequence[int]] = None,
                 pk_bytes: Optional[Sequence[bytes]] = None):
        self.pk_indices = list(pk_indices) if pk_indices is not None else None
        self.pk_bytes = list(pk_bytes) if pk_bytes is not None else None
        self.msg = bytes(msg)
        self.sig = bytes(sig)
        if (self.pk_indices is None) == (self.pk_bytes is None):
            raise ValueError("exactly one of pk_indices / pk_bytes")

    @property
    def n_pk(self):
        return len(self.pk_indices) if self.pk_indices is not None else len(self.pk_bytes)


class PackedSingleSets:
    """n single-pubkey sets over contiguous buffers (no per-set Python objects): set i has
    signing root msgs[32 i:32 i + 32], signature sigs[96 i:96 i + 96] and cached pubkey index
    idx[i].  For bulk shards (the config-5 epoch sweep: 2^20 sets) where SetSpec lists would
    cost seconds of host time.  `sets` / `nsets` / `slice(lo, hi)` feed bgv_verify_partial."""

    def __init__(self, msgs: bytes, sigs: bytes, idx: Sequence[int]):
        import numpy as np
        n = len(idx)
        if len(msgs) != 32 * n or len(sigs) != 96 * n:
            raise ValueError("msgs / sigs sizes do not match the index count")
        self._msg = np.frombuffer(bytes(msgs), dtype=np.uint8).copy()
        self._sig = np.frombuffer(bytes(sigs), dtype=np.uint8).copy()
        self._idx = np.asarray(idx, dtype=np.uint32).copy()
        rec = np.dtype([("n_pk", "<u4"), ("sig_len", "<u4"), ("pk_indices", "<u8"), ("pk_bytes", "<u8"),
                        ("msg", "<u8"), ("sig", "<u8")])
        assert rec.itemsize == ctypes.sizeof(BgvSet)
        arr = np.zeros(max(1, n), dtype=rec)
        k = np.arange(n, dtype=np.uint64)
        arr["n_pk"][:n] = 1
        arr["sig_len"][:n] = 96
        arr["pk_indices"][:n] = self._idx.ctypes.data + 4 * k
        arr["msg"][:n] = self._msg.ctypes.data + 32 * k
        arr["sig"][:n] = self._sig.ctypes.data + 96 * k
        self._arr = arr
        self.nsets = n

    def ptr(self, lo: int = 0):
        return ctypes.c_void_p(self._arr.ctypes.data + lo * ctypes.sizeof(BgvSet))


class PackedCall:
    """Keeps every buffer of one bgv_verify call alive and builds the C arrays."""

    def __init__(self, jobs):
        all_sets = []
        jarr = (BgvJob * max(1, len(jobs)))()
        for j, (sets, batchable) in enumerate(jobs):
            jarr[j].first_set = len(all_sets)
            jarr[j].n_sets = len(sets)
            jarr[j].batchable = 1 if batchable else 0
            all_sets.extend(sets)
        self.nsets = len(all_sets)
        sarr = (BgvSet * max(1, len(all_sets)))()
        keep = []
        for i, s in enumerate(all_sets):
            msg = ctypes.create_string_buffer(s.msg, 32) if len(s.msg) == 32 else None
            if msg is None:
                raise ValueError("signing root must be 32 bytes")
            sig = _buf(s.sig)
            keep += [msg, sig]
            sarr[i].n_pk = s.n_pk
            sarr[i].sig_len = len(s.sig)
            sarr[i].msg = ctypes.addressof(msg)
            sarr[i].sig = ctypes.addressof(sig)
            if s.pk_indices is not None:
                idx = (ctypes.c_uint32 * max(1, len(s.pk_indices)))(*s.pk_indices)
                keep.append(idx)
                sarr[i].pk_indices = ctypes.addressof(idx)
            else:
                pkb = _buf(b"".join(s.pk_bytes))
                keep.append(pkb)
                sarr[i].pk_bytes = ctypes.addressof(pkb)
        self.jobs, self.sets, self._keep = jarr, sarr, keep
