#!/bin/bash
# GPU-box parameter sweep of bench.py (one line per configuration).
set -o pipefail
mkdir -p gpurun_out
for dsp in ${DISPATCHERS:-2}; do for ms in ${MAXSLOTS:-131072}; do for inf in ${INFLIGHT:-16 32}; do
  BGV_DISPATCHERS=$dsp BGV_MAX_BATCH_SLOTS=$ms timeout -k 10 200 python bench.py --steps ${STEPS:-32} --warmup 1 --inflight $inf --no-cpu-baseline > gpurun_out/sw_d${dsp}_m${ms}_i${inf}.json 2>gpurun_out/sw.err || exit $?
  python tools/gpu/summarize.py gpurun_out/sw_d${dsp}_m${ms}_i${inf}.json
done; done; done
