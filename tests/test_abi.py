"""CPU checks of the drop-in boundary: libblsgpu.so builds for gfx950, loads, and
exports every function include/blsgpu.h declares.  No compute calls (no GPU here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "blsgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bgv_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ("bgv_init", "bgv_verify", "bgv_verify_async", "bgv_pubkeys_put", "bgv_aggregate_pubkeys",
                 "bgv_hash_to_g2", "bgv_strerror", "bgv_close"):
        assert must in fns


def test_library_exports_every_declared_symbol():
    from lodestar_amd import build, native
    lib_path = build.build(verbose=False)
    lib = ctypes.CDLL(lib_path)
    for fn in declared_functions():
        assert hasattr(lib, fn), fn
    assert set(native.EXPORTED_SYMBOLS) == set(declared_functions())
    # binding-level load (sets argtypes) and a pure host call
    L = native.load(lib_path)
    assert L.bgv_strerror(8) == b"BLST_INVALID_SIZE"
    assert L.bgv_strerror(-6) == b"BLST_PK_IS_INFINITY"
    assert L.bgv_strerror(32) == b"QUEUE_ABORTED"


def test_product_has_no_oracle_dependency():
    """The shipped package never imports the CPU oracle."""
    pkg = os.path.join(ROOT, "lodestar_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f


def test_chunkify_matches_reference():
    """beacon-node/test/unit/chain/bls/utils.test.ts"""
    from lodestar_amd.verifier import chunkify_maximize_chunk_size
    want = [[[0]], [[0, 1]], [[0, 1, 2]], [[0, 1, 2, 3]], [[0, 1, 2, 3, 4]],
            [[0, 1, 2], [3, 4, 5]], [[0, 1, 2, 3], [4, 5, 6]], [[0, 1, 2, 3], [4, 5, 6, 7]]]
    for i, w in enumerate(want):
        assert chunkify_maximize_chunk_size(list(range(i + 1)), 3) == w
