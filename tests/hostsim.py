"""ctypes wrapper over tests/native/libhostsim.so (host build of the device math).
Test infrastructure only."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "hostsim.cpp")
LIB = os.path.join(HERE, "native", "libhostsim.so")
CSRC = os.path.join(os.path.dirname(HERE), "lodestar_amd", "csrc")


def build(force=False):
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if not force and os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(d) for d in deps):
        return LIB
    # -DBGV_LAZY_CHECK: every lazy value (bls_lazy.h) is checked against its static bounds
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-DBGV_LAZY_CHECK", "-shared", "-fPIC", "-o", LIB, SRC])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
    return _lib


P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def fp_b(a):
    return (a % P).to_bytes(48, "big")


def b_fp(b):
    return int.from_bytes(b, "big")


def fp2_b(a):
    return fp_b(a[0]) + fp_b(a[1])


def b_fp2(b):
    return (b_fp(b[:48]), b_fp(b[48:96]))


def g2_b(pt):
    return fp2_b(pt[0]) + fp2_b(pt[1])


def b_g2(b):
    return (b_fp2(b[:96]), b_fp2(b[96:192]))


def g1_b(pt):
    return fp_b(pt[0]) + fp_b(pt[1])


def b_g1(b):
    return (b_fp(b[:48]), b_fp(b[48:96]))


def fp12_b_tower(tower_list):
    return b"".join(fp_b(x) for x in tower_list)


def b_fp12_tower(b):
    return [b_fp(b[48 * i:48 * i + 48]) for i in range(12)]


def buf(n):
    return ctypes.create_string_buffer(n)
