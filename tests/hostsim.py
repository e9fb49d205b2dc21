"""ctypes wrapper over tests/native/libhostsim.so (host build of the device math).
Test infrastructure only."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "hostsim.cpp")
CSRC = os.path.join(os.path.dirname(HERE), "lodestar_amd", "csrc")
# Two host builds of the same math: "wide" with the deferred-reduction Fp2 products the bulk
# kernel units use (bls_wide.h, -DBGV_LZ2_WIDE), "classic" with the fully reduced Karatsuba the
# other units use.
VARIANTS = {"wide": ["-DBGV_LZ2_WIDE"], "classic": []}
LIB = os.path.join(HERE, "native", "libhostsim.so")


def lib_path(variant="wide"):
    return LIB if variant == "wide" else os.path.join(HERE, "native", "libhostsim_%s.so" % variant)


def build(force=False, variant="wide"):
    out = lib_path(variant)
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    # -DBGV_LAZY_CHECK: every lazy value (bls_lazy.h) is checked against its static bounds
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-DBGV_LAZY_CHECK", "-shared", "-fPIC", "-o", out + ".tmp", SRC]
                          + VARIANTS[variant])
    os.replace(out + ".tmp", out)
    return out


_libs = {}


def lib(variant="wide"):
    if variant not in _libs:
        _libs[variant] = ctypes.CDLL(build(variant=variant))
    return _libs[variant]


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
