"""The bench's mainnet-shaped leg alone (config 4, one signing root per 128 sets), for A/Bs of the
uniform groups and the retry settings:

    python tools/gpu/mainnet_probe.py [REPEATS] [--corrupt F]

One JSON line per repeat (value in sets/s, the env knobs that were set).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("repeats", type=int, nargs="?", default=2)
    ap.add_argument("--nkeys", type=int, default=131072)
    ap.add_argument("--committee", type=int, default=128)
    ap.add_argument("--corrupt", type=float, default=0.01)
    ap.add_argument("--steps", type=int, default=64, help="calls timed per window")
    args = ap.parse_args()
    from lodestar_amd import native
    ctx = native.Context([0])
    ctx.keygen(b"".join(bench.interop_sk(i) for i in range(args.nkeys)), cache_first=0, want_pubkeys=False)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("BGV_")}
    for _ in range(args.repeats):
        r = bench.mainnet_shaped_throughput(ctx, native, args.nkeys, committee=args.committee, corrupt=args.corrupt,
                                            steps=args.steps)
        print(json.dumps({"mainnet_shaped": r["value"], "committee": args.committee, "corrupt": args.corrupt,
                          "steps": args.steps, "env": knobs}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
