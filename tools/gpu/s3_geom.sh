#!/bin/bash
# The driver's bench command (20/5 steps) at several super-batch sizes, and the retry fanout.
set -o pipefail
D=gpurun_out/s3/geom
mkdir -p $D
for round in 1 2; do
  for cpb in 20 10 5; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-block-import --calls-per-batch $cpb > $D/cpb${cpb}_$round.json 2> $D/cpb${cpb}_$round.err || { tail -3 $D/cpb${cpb}_$round.err; exit 1; }
    echo "cpb $cpb $(python tools/gpu/summarize.py $D/cpb${cpb}_$round.json)"
  done
  BGV_RETRY_FANOUT=4 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-block-import > $D/fan4_$round.json 2> $D/fan4_$round.err || { tail -3 $D/fan4_$round.err; exit 1; }
  echo "fanout4 $(python tools/gpu/summarize.py $D/fan4_$round.json)"
done
