#!/bin/bash
# Super-batch size (calls merged per device batch) on the default bench shape: STEPS timed calls,
# CPB in {16, 32, ...}; a window of >= 2 dispatcher periods needs STEPS >= 4 x CPB.
set -o pipefail
D=gpurun_out/s3/cpb
mkdir -p $D
for round in ${ROUNDS:-1 2 3}; do
  for b in ${CPBS:-16 32}; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-block-import --steps ${STEPS:-128} --calls-per-batch $b > $D/s${STEPS:-128}_b${b}_$round.json 2> $D/s${STEPS:-128}_b${b}_$round.err || { tail -3 $D/s${STEPS:-128}_b${b}_$round.err; exit 1; }
    python tools/gpu/summarize.py $D/s${STEPS:-128}_b${b}_$round.json
  done
done
