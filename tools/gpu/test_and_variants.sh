#!/bin/bash
# GPU parity tests first; then the variant comparison (tools/gpu/variants.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -n 3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/variants.sh
