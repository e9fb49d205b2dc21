"""Mainnet-shaped-roots probe: bench.mainnet_shaped_throughput alone (kernel traces of that
workload): python tools/gpu/mainnet_probe.py [committee=128]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from lodestar_amd import native  # noqa: E402

committee = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ctx = native.Context([0])
nkeys = 131072
ctx.keygen(b"".join(bench.interop_sk(i) for i in range(nkeys)), cache_first=0, want_pubkeys=False)
print(json.dumps(bench.mainnet_shaped_throughput(ctx, native, nkeys, committee=committee)))
ctx.close()
