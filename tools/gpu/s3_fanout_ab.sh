#!/bin/bash
# Retry fanout (BGV_RETRY_FANOUT) on the default bench (64/16 steps, 1 % corrupted), interleaved rounds.
set -o pipefail
D=gpurun_out/s3/fanout3
mkdir -p $D
for round in 1 2 3; do
  for f in ${FANOUTS:-8 4 2}; do
    BGV_RETRY_FANOUT=$f timeout -k 10 200 python bench.py --no-cpu-baseline --no-block-import > $D/f${f}_$round.json 2> $D/f${f}_$round.err || { tail -3 $D/f${f}_$round.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['device_groups_per_step'], round(d['call_device_ms'],1))" $D/f${f}_$round.json f$f
  done
done
