#!/bin/bash
# config-3 latency: wall p50 and a kernel trace of the same calls
set -o pipefail
mkdir -p gpurun_out/lat
export TMPDIR=/tmp
TAG=${TAG:-a}
timeout -k 10 200 python tools/gpu/latency_probe.py 30 > gpurun_out/lat/wall_$TAG.json 2> gpurun_out/lat/wall_$TAG.err || { tail -5 gpurun_out/lat/wall_$TAG.err; exit 1; }
cat gpurun_out/lat/wall_$TAG.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lat/tr_$TAG -o run --output-format csv -- python3 tools/gpu/latency_probe.py 30 > gpurun_out/lat/tr_$TAG.json 2> gpurun_out/lat/tr_$TAG.err || { tail -5 gpurun_out/lat/tr_$TAG.err; exit 1; }
f=$(find gpurun_out/lat/tr_$TAG -name "*kernel_trace.csv" | head -1)
python tools/gpu/trace_summary.py $f gpurun_out/lat/tr_$TAG.summary.json > /dev/null
python - <<PY
import json
d = json.load(open("gpurun_out/lat/tr_$TAG.summary.json"))
for k in d["kernels"][:14]:
    print(k["kernel"], k["grid_lanes"], k["launches"], k["median_ms"], k["total_ms"])
PY
