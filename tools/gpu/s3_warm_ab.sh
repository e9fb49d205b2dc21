#!/bin/bash
# Default bench with longer warmups / windows: is the 64/16 window's rate the sustained rate?
set -o pipefail
D=gpurun_out/s3/warm
mkdir -p $D
for round in 1 2; do
  for cfg in "64 16" "64 96" "64 256" "256 16" "20 5"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-block-import --steps $1 --warmup $2 > $D/s$1_w$2_$round.json 2> $D/s$1_w$2_$round.err || { tail -3 $D/s$1_w$2_$round.err; exit 1; }
    python tools/gpu/summarize.py $D/s$1_w$2_$round.json
  done
done
