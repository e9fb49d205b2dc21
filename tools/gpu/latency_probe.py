"""Config-3 latency probe: the bench's block-import call (131 sets, 16,898 cached keys) run
`runs` times back to back on an otherwise idle context; prints p50 / min wall ms.  Run under
`rocprofv3 --kernel-trace` to see which kernels make up one call's latency.

    python tools/gpu/latency_probe.py [runs=30]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from lodestar_amd import native  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    ctx = native.Context()
    nkeys = 16896 + 128
    ctx.keygen(b"".join(bench.interop_sk(i) for i in range(nkeys)), cache_first=0, want_pubkeys=False)
    r = bench.block_import_latency(ctx, native, nkeys, runs=runs)
    print(json.dumps(r))
    ctx.close()


if __name__ == "__main__":
    main()
