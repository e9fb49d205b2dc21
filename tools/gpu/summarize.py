"""One-line summary of bench.py JSON outputs (used by tools/gpu/record.sh).

    python tools/gpu/summarize.py FILE...     (FILE '-' reads JSON lines from stdin)
"""
import json
import sys


def lines(f):
    src = sys.stdin if f == "-" else open(f)
    for ln in src:
        ln = ln.strip()
        if ln.startswith("{"):
            yield f, json.loads(ln)


for f in sys.argv[1:]:
    for name, d in lines(f):
        r = d["roofline"]
        extra = []
        for k, lbl in (("block_import", "blk_p50"), ("mainnet_shaped_roots", "mainnet"),
                       ("aggregates_1024x128", "agg"), ("epoch_sweep", "sweep")):
            if k in d:
                v = d[k].get("p50_latency_ms") if k == "block_import" else round(d[k]["value"] / 1e6, 3)
                extra.append("%s %s" % (lbl, v))
        print(name.split("/")[-1], "steps %s/%s" % (d.get("steps"), d.get("timed_steps")), "value %.3fM" % (d["value"] / 1e6), "p50", round(d["p50_batch_latency_ms"], 1),
              "frac", round(r["frac"], 3), r.get("kernel", ""), "iso",
              {k: round(v, 2) for k, v in r.get("kernel_ms_isolated", {}).items()},
              "pf", round(r["pipeline_frac"], 3), " ".join(extra), flush=True)
