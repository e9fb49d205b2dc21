"""One-line summary of bench.py JSON outputs (used by the GPU sweep scripts)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f.split("/")[-1], round(d["value"]), "p50", round(d["p50_batch_latency_ms"], 1),
          "dev", round(d.get("call_device_ms", 0), 1), "wall", round(d.get("call_wall_ms", 0), 1),
          {k: round(v, 1) for k, v in d["kernel_ms_per_launch"].items()},
          "pf", round(d["roofline"]["pipeline_frac"], 3), flush=True)
