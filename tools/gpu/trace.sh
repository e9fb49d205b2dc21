#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
BGV_TRACE=1 BGV_DISPATCHERS=${D:-2} timeout -k 10 200 python bench.py --steps ${STEPS:-64} --warmup 1 --inflight ${INF:-32} --no-cpu-baseline > gpurun_out/trace.json 2> gpurun_out/trace.err || exit $?
python tools/gpu/summarize.py gpurun_out/trace.json; grep "\[bgv\]" gpurun_out/trace.err | tail -12
