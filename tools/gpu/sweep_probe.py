"""The bench's config-5 sweep leg alone (2^20 single sets, 2048 committee roots, one job as one
bgv_verify_partial + one final exponentiation), for A/Bs and BGV_TRACE breakdowns:

    python tools/gpu/sweep_probe.py [REPEATS]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    from lodestar_amd import native
    ctx = native.Context([0])
    barrier = bench.Barrier(1, 0)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("BGV_")}
    for _ in range(reps):
        r = bench.epoch_sweep(ctx, native, barrier, 0, 1)
        print(json.dumps({"sweep": r["value"], "ms": r["ms"], "env": knobs}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
