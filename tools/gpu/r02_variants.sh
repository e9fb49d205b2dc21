#!/bin/bash
# A/B of library variants on one box: isolated roofline call (per-kernel ms) and the
# driver's bench command, interleaved.
set -o pipefail
mkdir -p gpurun_out/var
for round in 1 2; do
  for v in base $VARIANTS; do
    lib=lodestar_amd/libblsgpu.so; [ $v != base ] && lib=lodestar_amd/libblsgpu_$v.so
    BLSGPU_LIB=$PWD/$lib timeout -k 10 120 python tools/gpu/roof_call.py > gpurun_out/var/roof_${v}_$round.json 2> gpurun_out/var/roof_${v}_$round.err || { tail -3 gpurun_out/var/roof_${v}_$round.err; exit 1; }
    echo "$v roof $(cat gpurun_out/var/roof_${v}_$round.json)"
  done
done
for v in base $VARIANTS; do
  lib=lodestar_amd/libblsgpu.so; [ $v != base ] && lib=lodestar_amd/libblsgpu_$v.so
  BLSGPU_LIB=$PWD/$lib timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-block-import > gpurun_out/var/bench_$v.json 2> gpurun_out/var/bench_$v.err || { tail -3 gpurun_out/var/bench_$v.err; exit 1; }
  echo "$v $(python tools/gpu/summarize.py gpurun_out/var/bench_$v.json)"
done
