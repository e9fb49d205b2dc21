#!/bin/bash
# sweep group size x retry fanout (dispatchers 2, 32 in flight, 64 steps)
set -o pipefail
mkdir -p gpurun_out
for gs in ${GS:-64 32 16}; do for f in ${FANOUTS:-8 64}; do
  BGV_GROUP_SLOTS=$gs BGV_RETRY_FANOUT=$f BGV_DISPATCHERS=${D:-2} timeout -k 10 200 python bench.py --steps ${STEPS:-64} --warmup 1 --inflight ${INF:-32} --no-cpu-baseline > gpurun_out/sw2_g${gs}_f${f}.json 2>gpurun_out/sw.err || exit $?
  python tools/gpu/summarize.py gpurun_out/sw2_g${gs}_f${f}.json
done; done
