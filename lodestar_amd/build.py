"""Build libblsgpu.so (HIP kernels for gfx950 + C-ABI host orchestration) in-tree.

    python -m lodestar_amd.build [--force]

The .so lands next to this file so it travels with the repository snapshot to
the GPU box (git-ignored, not gpurun-ignored).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libblsgpu.so")
# kernel translation units (compiled in parallel; each carries its own copy of the
# out-of-line arithmetic with its own register budget) and the host orchestration
KERNEL_UNITS = ["bgv_k_prep_bulk.hip", "bgv_k_miller_bulk.hip", "bgv_k_prep.hip", "bgv_k_prep_wave.hip", "bgv_k_miller.hip", "bgv_k_final.hip", "bgv_k_util.hip"]
SOURCES = [os.path.join(CSRC, f) for f in KERNEL_UNITS] + [os.path.join(CSRC, "bgv_api.cpp")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("BGV_OFFLOAD_ARCH", "gfx950")


def deps():
    out = list(SOURCES) + [os.path.join(HERE, "..", "include", "blsgpu.h")]
    out += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return out


def up_to_date(lib=LIB):
    return os.path.exists(lib) and all(os.path.getmtime(lib) >= os.path.getmtime(d) for d in deps())


OBJ_DIR = os.path.join(HERE, "..", "build", "obj")


def _headers():
    out = [os.path.join(HERE, "..", "include", "blsgpu.h")]
    return out + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]


def build(force=False, verbose=True, lib=LIB, defines=(), extra_flags=()):
    """defines: extra -D flags, extra_flags: extra compiler flags (A/B builds to another `lib`
    path: tools/ab_build.py; the product build takes neither).  Objects are
    cached per source under build/obj (the kernel unit takes minutes; the host unit seconds)
    and rebuilt when the source or any header is newer."""
    if not force and up_to_date(lib):
        return lib
    os.makedirs(OBJ_DIR, exist_ok=True)
    hdr_mtime = max(os.path.getmtime(h) for h in _headers())
    objs, procs = [], []
    extra_flags = list(extra_flags)
    tag = os.path.basename(lib) + ("." + "_".join(defines) if defines else "") + \
        ("." + str(abs(hash(" ".join(extra_flags)))) if extra_flags else "")
    for src in SOURCES:
        obj = os.path.join(OBJ_DIR, tag + "." + os.path.basename(src) + ".o")
        fresh = (not force and os.path.exists(obj)
                 and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime))
        if not fresh:
            cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
                   "-c", src, "-o", obj + ".tmp"] + ["-D" + d for d in defines] + extra_flags
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((subprocess.Popen(cmd), obj))
        objs.append(obj)
    for p, obj in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, "hipcc " + obj)
        os.replace(obj + ".tmp", obj)
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib + ".tmp"] + objs + ["-lpthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    return lib


NODE_DIR = os.path.join(HERE, "node")
NODE_SRC = os.path.join(NODE_DIR, "blsgpu_napi.c")
NODE_ADDON = os.path.join(NODE_DIR, "blsgpu.node")
NODE_INCLUDE = os.environ.get("NODE_INCLUDE", "/usr/include/node")


def build_node(force=False, verbose=True):
    """N-API addon (lodestar_amd/node/blsgpu.node) over libblsgpu.so; None when the image has
    no Node headers.  Built with gcc: the addon is plain C over the C-ABI."""
    if not os.path.exists(os.path.join(NODE_INCLUDE, "node_api.h")):
        return None
    build(verbose=verbose)
    srcs = [NODE_SRC, LIB, os.path.join(HERE, "..", "include", "blsgpu.h")]
    if not force and os.path.exists(NODE_ADDON) and all(
            os.path.getmtime(NODE_ADDON) >= os.path.getmtime(d) for d in srcs):
        return NODE_ADDON
    cmd = ["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-I" + NODE_INCLUDE, NODE_SRC, "-L" + HERE, "-lblsgpu",
           "-Wl,-rpath,$ORIGIN/..", "-o", NODE_ADDON + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(NODE_ADDON + ".tmp", NODE_ADDON)
    return NODE_ADDON


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_node(force="--force" in sys.argv)
