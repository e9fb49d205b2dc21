"""Build the CPU row of the Node gossip bench -- TEST INFRASTRUCTURE.

tests/node/blscpu.node: N-API binding (blscpu_napi.c) of oracle/cpu/libblscpu.so, the C++
restatement of the verify path; tests/node/blscpu_consts.bin: the SSWU / 3-isogeny constants
blscpu_init takes (288 + 1440 bytes, from oracle/bls12381.py, as oracle/cpu/blscpu.py passes
them).  Idempotent; prints the addon path.

    python tests/node/build_cpu.py
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import bls12381 as o  # noqa: E402
from oracle.cpu import blscpu  # noqa: E402

ADDON = os.path.join(HERE, "blscpu.node")
CONSTS = os.path.join(HERE, "blscpu_consts.bin")
NODE_INCLUDE = os.environ.get("NODE_INCLUDE", "/usr/include/node")


def _fp2b(a):
    return (a[0] % o.P).to_bytes(48, "big") + (a[1] % o.P).to_bytes(48, "big")


def build():
    lib = blscpu.build()
    src = os.path.join(HERE, "blscpu_napi.c")
    if not os.path.exists(ADDON) or os.path.getmtime(ADDON) < max(os.path.getmtime(src), os.path.getmtime(lib)):
        libdir = os.path.dirname(lib)
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-I" + NODE_INCLUDE, src, "-L" + libdir,
                               "-lblscpu", "-Wl,-rpath,$ORIGIN/../../oracle/cpu", "-o", ADDON + ".tmp"])
        os.replace(ADDON + ".tmp", ADDON)
    abz = b"".join(_fp2b(c) for c in (o.SSWU_A, o.SSWU_B, o.SSWU_Z))
    iso = b"".join(_fp2b(c) for k in ("xnum", "xden", "ynum", "yden") for c in o.ISO_CONSTANTS[k])
    assert len(abz) == 288 and len(iso) == 1440
    with open(CONSTS, "wb") as f:
        f.write(abz + iso)
    return ADDON


if __name__ == "__main__":
    print(build())
