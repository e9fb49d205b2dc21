#!/bin/bash
# Compare library variants (lodestar_amd/libblsgpu_<v>.so; "base" = libblsgpu.so):
# one 131072-set call at a time (clean per-kernel times), then the default bench.
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-base w2}; do
  if [ "$v" = base ]; then lib=lodestar_amd/libblsgpu.so; else lib=lodestar_amd/libblsgpu_$v.so; fi
  BLSGPU_LIB=$lib timeout -k 10 200 python bench.py --nsets 131072 --inflight 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/var_${v}_big.json 2> gpurun_out/var_${v}_big.err || exit $?
  python tools/gpu/summarize.py gpurun_out/var_${v}_big.json
  BLSGPU_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/var_${v}.json 2> gpurun_out/var_${v}.err || exit $?
  python tools/gpu/summarize.py gpurun_out/var_${v}.json
done
