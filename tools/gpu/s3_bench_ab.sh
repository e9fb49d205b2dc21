#!/bin/bash
# A/B of library variants on the default bench (64/16 steps, no CPU baseline / extras), two rounds.
set -o pipefail
mkdir -p gpurun_out/s3/bench_ab
for round in 1 2; do
  for v in base $VARIANTS; do
    lib=lodestar_amd/libblsgpu.so; [ $v != base ] && lib=lodestar_amd/libblsgpu_$v.so
    BLSGPU_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-block-import > gpurun_out/s3/bench_ab/${v}_$round.json 2> gpurun_out/s3/bench_ab/${v}_$round.err || { tail -3 gpurun_out/s3/bench_ab/${v}_$round.err; exit 1; }
    echo "$v $(python tools/gpu/summarize.py gpurun_out/s3/bench_ab/${v}_$round.json)"
  done
done
