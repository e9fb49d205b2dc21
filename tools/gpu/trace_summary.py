"""Per-kernel summary of a rocprofv3 --kernel-trace CSV: launches grouped by grid size
(slots), mean / median duration, and the busy-time union of all kernels.

    python tools/gpu/trace_summary.py <kernel_trace.csv> [out.json]
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    by = defaultdict(list)
    spans = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        b, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) * int(r.get("Grid_Size_Y", 1) or 1)
        by[(name, grid)].append((e - b) / 1e6)
        spans.append((b, e))
    spans.sort()
    busy, cur_b, cur_e = 0, None, None
    for b, e in spans:
        if cur_e is None or b > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_b
            cur_b, cur_e = b, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_b
    out = {"wall_ms": (spans[-1][1] - spans[0][0]) / 1e6 if spans else 0, "busy_ms": busy / 1e6, "kernels": []}
    for (name, grid), d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        out["kernels"].append({"kernel": name, "grid_lanes": grid, "launches": len(d), "total_ms": round(sum(d), 3),
                               "mean_ms": round(statistics.mean(d), 3), "median_ms": round(statistics.median(d), 3),
                               "min_ms": round(min(d), 3), "max_ms": round(max(d), 3)})
    txt = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt)
    for k in out["kernels"][:24]:
        print("%-24s grid %8d  n %4d  total %9.1f  mean %8.3f  med %8.3f  min %8.3f  max %8.3f" % (
            k["kernel"], k["grid_lanes"], k["launches"], k["total_ms"], k["mean_ms"], k["median_ms"], k["min_ms"],
            k["max_ms"]))
    print("wall %.1f ms  busy %.1f ms" % (out["wall_ms"], out["busy_ms"]))


if __name__ == "__main__":
    main()
