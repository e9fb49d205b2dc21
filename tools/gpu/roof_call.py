"""The bench's roofline measurement alone (bench.roofline_isolated): one 64,512-set verify
call (k_miller = one wave per SIMD), repeated, on an idle device.  Driver for the PMC
passes of tools/gpu/pmc.sh and the `roof` step of tools/gpu/record.sh."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from lodestar_amd import native  # noqa: E402

ctx = native.Context([0])
nkeys = 131072
ctx.keygen(b"".join(bench.interop_sk(i) for i in range(nkeys)), cache_first=0, want_pubkeys=False)
print(json.dumps(bench.roofline_isolated(ctx, native, nkeys)))
ctx.close()
