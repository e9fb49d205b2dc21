#!/bin/bash
# k_miller translation-unit variants (lodestar_amd/libblsgpu_<v>.so): GPU parity with each,
# then tools/gpu/variants.sh over VARIANTS, then a kernel trace per variant (VGPR / AGPR / scratch).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS}; do
  [ "$v" = base ] && continue
  BLSGPU_LIB=lodestar_amd/libblsgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${v}_pytest.log 2>&1 || { tail -20 gpurun_out/${v}_pytest.log; exit 1; }
  tail -1 gpurun_out/${v}_pytest.log
done
bash tools/gpu/variants.sh || exit 1
for v in ${VARIANTS}; do
  [ "$v" = base ] && continue
  BLSGPU_LIB=lodestar_amd/libblsgpu_$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${v}_trace -o run --output-format csv -- python bench.py --nsets 65536 --inflight 1 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2>gpurun_out/${v}_trace.err || exit 1
done
