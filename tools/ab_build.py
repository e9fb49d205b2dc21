"""A/B tooling, not the product build: libblsgpu with extra -D defines (and compiler flags from
BGV_VARIANT_FLAGS) built to lodestar_amd/libblsgpu_NAME.so, loaded with BLSGPU_LIB=... by the
bench or the tests (tools/gpu/ab.sh).

    python tools/ab_build.py NAME [DEFINE ...]      e.g.  python tools/ab_build.py w2 BGV_WPE_BULK=2
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lodestar_amd import build as b  # noqa: E402

if __name__ == "__main__":
    name, defs = sys.argv[1], sys.argv[2:]
    flags = os.environ.get("BGV_VARIANT_FLAGS", "").split()
    print(b.build(force=True, lib=os.path.join(b.HERE, "libblsgpu_%s.so" % name), defines=defs, extra_flags=flags))
