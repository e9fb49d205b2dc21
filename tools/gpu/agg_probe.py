"""Config-2 probe: the bench's aggregate-set throughput measurement alone (for a kernel
trace of that workload: python tools/gpu/agg_probe.py [calls] [inflight])."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from lodestar_amd import native  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 512
inflight = int(sys.argv[2]) if len(sys.argv) > 2 else 128
ctx = native.Context([0])
nkeys = 131072
ctx.keygen(b"".join(bench.interop_sk(i) for i in range(nkeys)), cache_first=0, want_pubkeys=False)
print(json.dumps(bench.aggregate_throughput(ctx, native, nkeys, calls=calls, inflight=inflight)))
ctx.close()
