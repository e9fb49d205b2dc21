#!/bin/bash
# super-batch geometry sweep of the steady-state bench (driver's --steps 20 --warmup 5)
set -o pipefail
mkdir -p gpurun_out/sweep
for B in 5 10 16 20; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-block-import --calls-per-batch $B > gpurun_out/sweep/b$B.json 2> gpurun_out/sweep/b$B.err || { tail -3 gpurun_out/sweep/b$B.err; exit 1; }
  python tools/gpu/summarize.py gpurun_out/sweep/b$B.json
done
for B in 16 20; do
  BGV_DISPATCHERS=3 timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-block-import --calls-per-batch $B > gpurun_out/sweep/d3b$B.json 2> gpurun_out/sweep/d3b$B.err || { tail -3 gpurun_out/sweep/d3b$B.err; exit 1; }
  python tools/gpu/summarize.py gpurun_out/sweep/d3b$B.json
done
timeout -k 10 150 python bench.py --steps 80 --warmup 20 --no-cpu-baseline --no-block-import --calls-per-batch 20 > gpurun_out/sweep/long20.json 2> gpurun_out/sweep/long20.err || exit 1
python tools/gpu/summarize.py gpurun_out/sweep/long20.json
