#!/bin/bash
# GPU-box quick check: parity tests, then the default bench without the CPU baseline.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-q}
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python tools/gpu/summarize.py gpurun_out/bench_$TAG.json
