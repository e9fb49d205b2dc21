#!/bin/bash
# A/B of library variants on the config-2 workload (tools/gpu/agg_probe.py) and the isolated
# roofline call.  VARIANTS="a1 a4" -> lodestar_amd/libblsgpu_<v>.so; base = libblsgpu.so.
set -o pipefail
mkdir -p gpurun_out/s3/agg_ab
for round in 1 2; do
  for v in base $VARIANTS; do
    lib=lodestar_amd/libblsgpu.so; [ $v != base ] && lib=lodestar_amd/libblsgpu_$v.so
    BLSGPU_LIB=$PWD/$lib timeout -k 10 200 python tools/gpu/agg_probe.py 1024 128 > gpurun_out/s3/agg_ab/${v}_$round.json 2> gpurun_out/s3/agg_ab/${v}_$round.err || { tail -3 gpurun_out/s3/agg_ab/${v}_$round.err; exit 1; }
    echo "$v agg $(cat gpurun_out/s3/agg_ab/${v}_$round.json | python -c 'import json,sys; print(round(json.load(sys.stdin)["value"]))')"
  done
done
