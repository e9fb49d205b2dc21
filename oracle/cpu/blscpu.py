"""ctypes wrapper of oracle/cpu/libblscpu.so — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

The C++ restatement of the verify path (blscpu.cpp) with a BlsMultiThreadWorkerPool
style thread pool.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it.  Curve constants (SSWU, 3-isogeny) are passed in from the
Python oracle at load time.
"""
import ctypes
import os
import subprocess

from oracle import bls12381 as o

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libblscpu.so")


def build(force=False):
    src = os.path.join(HERE, "blscpu.cpp")
    if force or not os.path.exists(LIB) or any(os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, f))
                                             for f in ("blscpu.cpp", "fp_mulx.h", "Makefile")):
        subprocess.check_call(["make", "-s", "-C", HERE] + (["-B"] if force else []))
    return LIB


_lib = None


def _fp2b(a):
    return (a[0] % o.P).to_bytes(48, "big") + (a[1] % o.P).to_bytes(48, "big")


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(build())
        abz = b"".join(_fp2b(c) for c in (o.SSWU_A, o.SSWU_B, o.SSWU_Z))
        iso = b"".join(_fp2b(c) for k in ("xnum", "xden", "ynum", "yden") for c in o.ISO_CONSTANTS[k])
        assert len(iso) == 15 * 96
        L.blscpu_init(abz, iso)
        L.blscpu_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                    ctypes.c_void_p]
        _lib = L
    return _lib


def hash_to_g2(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(192)
    assert lib().blscpu_hash_to_g2(msg, len(msg), out) == 1
    return out.raw


def sk_to_pk96(sks32: bytes) -> bytes:
    n = len(sks32) // 32
    out = ctypes.create_string_buffer(96 * max(1, n))
    lib().blscpu_sk_to_pk96(sks32, ctypes.c_size_t(n), out)
    return out.raw[:96 * n]


def verify_jobs(jobs, mode=0, threads=1, seed=0x1234):
    """jobs: list of (sets, batchable), sets = [(pk96_affine_uncompressed, msg32, sig_bytes)];
    a pk of None is an aggregate of zero pubkeys, rejected on the main thread with
    EMPTY_AGGREGATE_ARRAY before any job runs (chain/bls/utils.ts:11).
    Returns per-job codes (1, 0, -code)."""
    empty = [any(p is None for p, _, _ in sets) for sets, _ in jobs]
    jobs = [([(p or b"\x40" + bytes(95), m, s) for p, m, s in sets], b) for sets, b in jobs]
    pk, msgs, sigs, lens, triples = [], [], [], [], []
    n = 0
    for sets, batchable in jobs:
        triples += [n, len(sets), 1 if batchable else 0]
        for p, m, s in sets:
            pk.append(p)
            msgs.append(m)
            sigs.append(s[:96].ljust(96, b"\0"))
            lens.append(len(s))
            n += 1
    U32 = ctypes.c_uint32
    out = (ctypes.c_int32 * max(1, len(jobs)))()
    lib().blscpu_verify(b"".join(pk) or b"\0", b"".join(msgs) or b"\0", b"".join(sigs) or b"\0",
                        (U32 * max(1, n))(*lens), (U32 * max(1, len(triples)))(*triples), len(jobs), mode,
                        threads, seed, out)
    return [-20 if e else c for e, c in zip(empty, out[:len(jobs)])]
