#!/bin/bash
# kernel traces of the driver's bench command (1 % and 0 % corruption)
set -o pipefail
mkdir -p gpurun_out/trace
export TMPDIR=/tmp
for C in 0.01 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trace/c$C -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-block-import --corrupt $C > gpurun_out/trace/c$C.json 2> gpurun_out/trace/c$C.err || { tail -5 gpurun_out/trace/c$C.err; exit 1; }
  python tools/gpu/summarize.py gpurun_out/trace/c$C.json
  f=$(find gpurun_out/trace/c$C -name "*kernel_trace.csv" | head -1)
  python tools/gpu/trace_summary.py $f gpurun_out/trace/c$C.summary.json
done
